// nfk_fused_chain2.hip -- the chained fused NSF_CL launch (nfk_fused_nsf_chain,
// nf/models.py:13-40 over nf/flows.py:227-253 layers) with TWO 16-sample
// tiles per wave.
//
// Same pack, sub-record stream (NfkSplit), arithmetic and per-layer order as
// k_fused_nsf<..., SPLIT, CHAIN> (nfk_fused_impl.h), so z, log|det| and
// log_prob are bitwise those of that kernel; what changes is the work per
// wave: every A fragment read from the LDS slot feeds the MFMAs of both
// sample tiles (half the ds_read_b128 and half the LDS-DMA bytes per sample),
// the two tiles' epilogues are independent instruction streams the scheduler
// can interleave, and a workgroup barrier covers 128 samples.  256 VGPRs,
// two waves per SIMD (two 4-wave workgroups per CU, 77 KiB of LDS each):
// 2048 wave slots x 32 samples, so 2^17 rows (the 8-GPU strong-scaling
// shard) are exactly two rounds where the 16-sample form fills 2.67.
// Schedule: whole-record phases (no pipelined chunk schedule).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "nfk_fused_impl.h"


namespace nfk_fused {

constexpr int kC2Tiles = 2;  // sample tiles per wave

// gemm_h with NTL sample tiles sharing every A fragment: acc[s][T0 .. T0 + NT)
template <int KBH, bool T1, int NT, int NS, int T0, int NA>
__device__ __forceinline__ void gemm_h2(const h8 (&bh)[kC2Tiles][KBH], const h8 (&bl)[kC2Tiles][KBH],
                                        const h4 (&btail)[kC2Tiles], const float4* slot, int lane,
                                        f32x4 (&acc)[kC2Tiles][NA]) {
    constexpr int NPR = (NT + 1) / 2;
    constexpr int N = KBH * NPR;
    constexpr int NI = N + (T1 ? NPR : 0);
    constexpr int NTG = T1 ? (NS + 1) / 2 : 0;
    const int q = lane >> 4;
    const float4* tail = slot + KBH * NS * 2 * 64;
    const float4* bias = tail + NTG * 64;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const f32x4 b = as_f32x4(bias[(T0 + t) * 4 + q]);
#pragma unroll
        for (int s = 0; s < kC2Tiles; ++s) acc[s][T0 + t] = b;
    }
    auto fetch = [&](int i, float4 (&r)[4]) {
        if (i < N) {
            const int kb = i / NPR, pr = i - kb * NPR;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (2 * pr + (j >> 1) < NT) r[j] = slot[((kb * NS + 2 * pr) * 2 + j) * 64 + lane];
        } else {
            r[0] = tail[(i - N) * 64 + lane];
        }
    };
    float4 ring[2][4];
    fetch(0, ring[0]);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int pr = i < N ? i % NPR : i - N, kb = i < N ? i / NPR : 0, t0 = T0 + 2 * pr;
        const bool two = t0 + 1 < T0 + NT;
        if (i + 1 < NI) fetch(i + 1, ring[(i + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        const float4* r = ring[i & 1];
        if (i >= N) {  // tail step (T1)
            if (i == N && NT <= 2) {
                // (gemm_h: a 16x16x16 MFMA reading what a 16x16x32 MFMA one
                // instruction earlier wrote is not forwarded; the second tile's
                // MFMAs separate them here only partly, so wait as gemm_h does)
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_nop 7\n\ts_nop 7");
                __builtin_amdgcn_sched_barrier(0);
            }
            const float4 w = r[0];
            const h4 a0 = __builtin_bit_cast(h4, make_float2(w.x, w.y)), a1 = __builtin_bit_cast(h4, make_float2(w.z, w.w));
#pragma unroll
            for (int s = 0; s < kC2Tiles; ++s) {
                acc[s][t0] = mfma16k16(a0, btail[s], acc[s][t0]);
                if (two) acc[s][t0 + 1] = mfma16k16(a1, btail[s], acc[s][t0 + 1]);
            }
            continue;
        }
        const h8 ahi0 = __builtin_bit_cast(h8, r[0]), alo0 = __builtin_bit_cast(h8, r[1]);
        const h8 ahi1 = __builtin_bit_cast(h8, r[2]), alo1 = __builtin_bit_cast(h8, r[3]);
        // products in gemm_h's order per accumulator (lo.hi, hi.lo, hi.hi), the
        // four (tile, sample tile) accumulators interleaved
#pragma unroll
        for (int s = 0; s < kC2Tiles; ++s) {
            acc[s][t0] = mfma16(alo0, bh[s][kb], acc[s][t0]);
            if (two) acc[s][t0 + 1] = mfma16(alo1, bh[s][kb], acc[s][t0 + 1]);
        }
#pragma unroll
        for (int s = 0; s < kC2Tiles; ++s) {
            acc[s][t0] = mfma16(ahi0, bl[s][kb], acc[s][t0]);
            if (two) acc[s][t0 + 1] = mfma16(ahi1, bl[s][kb], acc[s][t0 + 1]);
        }
#pragma unroll
        for (int s = 0; s < kC2Tiles; ++s) {
            acc[s][t0] = mfma16(ahi0, bh[s][kb], acc[s][t0]);
            if (two) acc[s][t0 + 1] = mfma16(ahi1, bh[s][kb], acc[s][t0 + 1]);
        }
    }
}

template <int KBH, bool T1, int NT, int NS, int J, class Step>
__device__ __forceinline__ void gemm_parts2(const h8 (&bh)[kC2Tiles][KBH], const h8 (&bl)[kC2Tiles][KBH],
                                            const h4 (&btail)[kC2Tiles], const float4* slot, int lane,
                                            f32x4 (&acc)[kC2Tiles][NT], Step&& step) {
    constexpr int T0 = J * NS;
    constexpr int N = (NT - T0) < NS ? (NT - T0) : NS;
    constexpr bool last = T0 + NS >= NT;
    gemm_h2<KBH, T1, N, NS, T0, NT>(bh, bl, btail, slot, lane, acc);
    step(last);
    if constexpr (!last) gemm_parts2<KBH, T1, NT, NS, J + 1>(bh, bl, btail, slot, lane, acc, step);
}

// LDS of one workgroup: the sub-record slot, the status words and byte maps,
// each wave's kC2Tiles x [16][D + 1] row tiles, each wave's kC2Tiles bin
// lookup tables
// byte maps of the chain: nl layers' input columns + the output map (+ the
// training form's nl - 1 saved-input maps)
__host__ __device__ inline int chain2_map_bytes(int nl, int D, bool saved) {
    return (nl + 1) * D + (saved ? (nl - 1) * D : 0);
}

inline size_t lds_bytes_chain2(const Layout& L, int nl, bool saved = false) {
    const int D = L.n_lo + L.n_up;
    return (size_t)split_slot_blocks(L) * 1024 + (size_t)((4 * nl + chain2_map_bytes(nl, D, saved) + 15) / 16) * 16 +
           (size_t)kNsfWaves * kC2Tiles * 16 * (D + 1) * sizeof(float) +
           (size_t)kNsfWaves * kC2Tiles * L.K * 64 * sizeof(int);
}

template <int KBH, bool T1, int K, bool INV>
__global__ __launch_bounds__(64 * kNsfWaves, 2) void k_nsf_chain2(FusedArgs a) {
    using ArgsK = const __attribute__((address_space(4))) FusedArgs;
    ArgsK* A = (ArgsK*)__builtin_amdgcn_kernarg_segment_ptr();
    (void)a;
    constexpr int NTL = kC2Tiles;
    constexpr int HT = 2 * KBH + (T1 ? 1 : 0);
    constexpr int DN = K - 1 > 0 ? K - 1 : 1;
    using SP = NfkSplit<KBH, T1, K, HT>;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4, sl = lane & 15;
    const int D = A->n_lo + A->n_up;
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    float4* slot = lds4;
    const int NL = A->nlayers;
    int32_t* const cst = reinterpret_cast<int32_t*>(lds4 + A->slot_blocks * 64);
    uint8_t* const cm = reinterpret_cast<uint8_t*>(cst + NL);
    const uint8_t* c_lo = cm;
    const uint8_t* c_up = cm;
    const uint8_t* const c_src = cm + NL * D;
    const bool saved = A->saves != nullptr;
    const uint8_t* const c_sav = cm + (NL + 1) * D;  // training form: saved-input maps
    const int XS = D + 1;
    float* const xbase =
        reinterpret_cast<float*>(lds4 + A->slot_blocks * 64 + (4 * NL + chain2_map_bytes(NL, D, saved) + 15) / 16);
    float* const xt = xbase + wid * NTL * 16 * XS;  // this wave's NTL row tiles
    int* const scr = reinterpret_cast<int*>(xbase + kNsfWaves * NTL * 16 * XS) + wid * NTL * K * 64;
    const float* pk = A->packs[0];
    int lyr = 0;
    const int offA = INV ? A->blk_w : 0, offB = INV ? 0 : A->blk_w, offC = 2 * A->blk_w;
    const int64_t b0 = ((int64_t)blockIdx.x * kNsfWaves + wid) * 16 * NTL;
    int nrows[NTL];
    bool row_ok[NTL];
#pragma unroll
    for (int s = 0; s < NTL; ++s) {
        const int64_t rem = A->batch - (b0 + 16 * s);
        nrows[s] = rem <= 0 ? 0 : (rem < 16 ? (int)rem : 16);
        row_ok[s] = sl < nrows[s];
    }
    const int nall = nrows[0] + nrows[1];
    h8 bh[NTL][KBH], bl[NTL][KBH];
    h4 btail[NTL];
#pragma unroll
    for (int s = 0; s < NTL; ++s) btail[s] = h4{0, 0, 0, 0};

    const int NSR = 1 + SP::NH2 + A->NCH * SP::SPC;
    int sr = 0;
    auto gemm_end = [&](bool last) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (sr + 1 < NSR) {
            stage_split<KBH, T1, K, HT>(a, pk, sr + 1, offA, offB, offC, slot, wid, lane);
        } else if (lyr + 1 < NL) {
            stage_split<KBH, T1, K, HT>(a, A->packs[lyr + 1], 0, offA, offB, offC, slot, wid, lane);
        }
        ++sr;
        if (!last) {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
    };
    auto epi_end = [&]() {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    auto gemm_rec = [&](auto& acc) {
        constexpr int N = sizeof(acc[0]) / sizeof(f32x4);
        gemm_parts2<KBH, T1, N, SP::NS, 0>(bh, bl, btail, slot, lane, acc, gemm_end);
    };

    // ---- prologue: the log|det| being accumulated (mode 2; a plain load
    // before any DMA is in flight), whole x rows of both tiles (rows past the
    // batch re-read row 0 of the wave), the first layer-1 record, the byte maps
    float ld_acc[NTL];
#pragma unroll
    for (int s = 0; s < NTL; ++s)
        ld_acc[s] = (q == 0 && row_ok[s] && A->mode == 2) ? A->logdet[b0 + 16 * s + sl] : 0.0f;
    if (nall > 0) {
        const uint32_t base = lds_addr(xt);
        for (int r = 0; r < 16 * NTL; ++r) {
            // padding rows of a tile copy its first row (the one-tile kernel's
            // choice: the tile's layer-1 scale, a max over its rows, unchanged)
            const int t0 = r & ~15;
            const float* src = A->x + (b0 + (r < nall ? r : (t0 < nall ? t0 : 0))) * A->ldx;
            for (int c0 = 0; c0 < D; c0 += 64)
                if (c0 + lane < D) {
#if NFK_X_NT
                    dma4_nt(src + c0 + lane, base + (r * XS + c0) * 4);
#else
                    dma4(src + c0 + lane, base + (r * XS + c0) * 4);
#endif
                }
        }
    }
    stage_split<KBH, T1, K, HT>(a, pk, 0, offA, offB, offC, slot, wid, lane);
    for (int i = threadIdx.x; i < (NL + 1) * D; i += 64 * kNsfWaves) cm[i] = (uint8_t)A->cmaps[i];
    if (saved)
        for (int i = threadIdx.x; i < (NL - 1) * D; i += 64 * kNsfWaves) cm[(NL + 1) * D + i] = (uint8_t)A->smaps[i];
    if ((int)threadIdx.x < NL) cst[threadIdx.x] = 0;
    dma_barrier();

    for (int l = 0; l < NL; ++l) {
        asm volatile("" : "+s"(A));
        lyr = l;
        pk = A->packs[l];
        c_lo = cm + l * D;
        c_up = c_lo + A->n_lo;
        sr = 0;
        const FusedConst c = *(const FusedConst*)&A->c;  // by value: SGPRs for the layer
        const float un1 = pk[3], un2 = pk[4], un3 = pk[5];
        bool any_in = false, any_nd = false;
        if (saved && l > 0) {
            // training form: this layer's input (the previous layer's z, in its
            // own column order) for the layer's backward; the tile's last writes
            // are this wave's own, retired at the barrier that ended the layer
            const uint8_t* sm = c_sav + (l - 1) * D;
            float* dst = A->saves + (int64_t)(l - 1) * A->save_stride;
            for (RowWalk w(lane, D >> 2); w.r < nall; w.next()) {
                const float* row = xt + w.r * XS;
                const int o = 4 * w.k;
                *reinterpret_cast<float4*>(dst + (b0 + w.r) * A->ld_saves + o) =
                    make_float4(row[sm[o]], row[sm[o + 1]], row[sm[o + 2]], row[sm[o + 3]]);
            }
        }

        // ---- layer 1 (nfk_fused_impl.h phase 0, per sample tile: the tile's
        // power-of-two input scale)
        {
            f32x4 h1[NTL][HT];
            float unx[NTL];
            h8 xh[NTL], xl8[NTL];
#pragma unroll
            for (int s = 0; s < NTL; ++s) {
                const float* xr = xt + (16 * s + sl) * XS;
                float e[8];
                if (A->n_lo >= 32) {  // (uniform) every lane group's 8 inputs exist: plain reads
#pragma unroll
                    for (int j = 0; j < 8; ++j) e[j] = xr[c_lo[8 * q + j]];
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int k = 8 * q + j;
                        const bool ok = k < A->n_lo;  // unconditional reads, then selected
                        const float v = xr[c_lo[ok ? k : 0]];
                        e[j] = ok ? v : 0.0f;
                    }
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
                unx[s] = ldexpf(un1, ex - 14);
                const float bsc = ldexpf(1.0f, 14 - ex) / un1;
                const float4* bias = slot + A->KB1 * HT * 2 * 64;
#pragma unroll
                for (int t = 0; t < HT; ++t) {
                    const float4 bv = bias[t * 4 + q];
                    h1[s][t] = f32x4{bv.x * bsc, bv.y * bsc, bv.z * bsc, bv.w * bsc};
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float v = e[j] * sx;
                    const _Float16 hh = (_Float16)v;
                    xh[s][j] = hh;
                    xl8[s][j] = (_Float16)(v - (float)hh);
                }
            }
#pragma unroll
            for (int t = 0; t < HT; ++t) {
                const h8 ahi = __builtin_bit_cast(h8, slot[(t * 2) * 64 + lane]);
                const h8 alo = __builtin_bit_cast(h8, slot[(t * 2 + 1) * 64 + lane]);
#pragma unroll
                for (int s = 0; s < NTL; ++s) {
                    h1[s][t] = mfma16(alo, xh[s], h1[s][t]);
                    h1[s][t] = mfma16(ahi, xl8[s], h1[s][t]);
                    h1[s][t] = mfma16(ahi, xh[s], h1[s][t]);
                }
            }
            gemm_end(true);
#pragma unroll
            for (int s = 0; s < NTL; ++s) act_operands<KBH, T1, HT>(h1[s], -2.0f * kL2E * unx[s], bh[s], bl[s], btail[s]);
        }
        epi_end();
        {
            f32x4 h2[NTL][HT];
            gemm_rec(h2);
#pragma unroll
            for (int s = 0; s < NTL; ++s) act_operands<KBH, T1, HT>(h2[s], -2.0f * kL2E * un2, bh[s], bl[s], btail[s]);
        }
        epi_end();

        const float l2e3 = kL2E * un3;
        float ldsum[NTL] = {0.0f, 0.0f};
        int jj4[4];
        float xv[NTL][4];
        int kb[NTL][4];
        float cw_k[NTL][4], w_k[NTL][4], ch_k[NTL][4], h_k[NTL][4];
        for (int ch = 0; ch < A->NCH; ++ch) {
            const int jbase = 16 * ch;
            {
                f32x4 acc[NTL][K];
                gemm_rec(acc);
                // map reads and x reads unconditional (a guarded read became a
                // branch with its own LDS round trip per coordinate)
                // (uniform) n_up a multiple of 16: every chunk's coordinates exist
                const bool full_up = (A->n_up & 15) == 0;
                int tc4[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    jj4[r] = jbase + 4 * q + r;
                    const bool ok = full_up || jj4[r] < A->n_up;
                    tc4[r] = full_up ? (int)c_up[jj4[r]] : (ok ? (int)c_up[ok ? jj4[r] : 0] : D);
                }
#pragma unroll
                for (int s = 0; s < NTL; ++s) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float v = xt[(16 * s + sl) * XS + tc4[r]];
                        xv[s][r] = (full_up || jj4[r] < A->n_up) ? v : 0.0f;
                    }
                    knot_phase<K, true, 0, 4, true>(acc[s], xv[s], c, l2e3, kb[s], INV ? ch_k[s] : cw_k[s],
                                                   INV ? h_k[s] : w_k[s], scr + s * K * 64, lane);
                }
            }
            epi_end();
            {
                f32x4 acc[NTL][K];
                gemm_rec(acc);
#pragma unroll
                for (int s = 0; s < NTL; ++s)
                    knot_phase<K, false, 0, 4, true>(acc[s], xv[s], c, l2e3, kb[s], INV ? cw_k[s] : ch_k[s],
                                                    INV ? w_k[s] : h_k[s], scr + s * K * 64, lane);
            }
            epi_end();
            {
                f32x4 accd[NTL][DN];
                gemm_rec(accd);
#pragma unroll
                for (int s = 0; s < NTL; ++s) {
                    float* fs = reinterpret_cast<float*>(scr + s * K * 64);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        // epilogue C of k_fused_nsf, op for op
                        const int k = kb[s][r];
                        float raw_k = accd[s][0][r], raw_k1 = accd[s][0][r];
#pragma unroll
                        for (int j = 0; j < K - 1; ++j) fs[j * 64 + lane] = accd[s][j][r];
                        raw_k = fs[(k > 0 ? k - 1 : 0) * 64 + lane];
                        raw_k1 = fs[(k < K - 1 ? k : K - 2) * 64 + lane];
                        const float dv_k = nfk_deriv_lean_s(raw_k, l2e3, c.min_d);
                        const float dv_k1 = nfk_deriv_lean_s(raw_k1, l2e3, c.min_d);
                        const float d_k = (k == 0) ? c.d_edge : dv_k;
                        const float d_k1 = (k == K - 1) ? c.d_edge : dv_k1;
                        const float x = xv[s][r];
                        const float rw = nfk_rcp_fast(w_k[s][r]);
                        const float delta = h_k[s][r] * rw;
                        const float gap = (d_k + d_k1) - 2.0f * delta;
                        float out, th;
                        bool nd = false;
                        if (INV) {
                            const float y = x - ch_k[s][r];
                            const float qa = y * gap + h_k[s][r] * (delta - d_k);
                            const float qb = h_k[s][r] * d_k - y * gap;
                            const float qc = (-delta) * y;
                            const float disc = qb * qb - (4.0f * qa) * qc;
                            nd = !(disc >= 0.0f);
                            const float root = nfk_div<true>(2.0f * qc, -qb - sqrtf(disc));
                            out = root * w_k[s][r] + cw_k[s][r];
                            th = root;
                        } else {
                            th = (x - cw_k[s][r]) * rw;
                        }
                        const float t1mt = th * (1.0f - th);
                        const float den = delta + gap * t1mt;
                        if (!INV) {
                            const float num = h_k[s][r] * (delta * (th * th) + d_k * t1mt);
                            out = ch_k[s][r] + nfk_div<true>(num, den);
                        }
                        const float omt = 1.0f - th;
                        const float dnum =
                            (delta * delta) * ((d_k1 * (th * th) + (2.0f * delta) * t1mt) + d_k * (omt * omt));
                        float lad = (__builtin_amdgcn_logf(dnum) - 2.0f * __builtin_amdgcn_logf(den)) * kLN2;
                        lad = INV ? -lad : lad;
                        const bool inside = (x >= c.lo) && (x <= c.hi);
                        const bool live = jj4[r] < A->n_up && row_ok[s];
                        out = inside ? out : x;
                        // past n_up: the padding column (the map re-read: the
                        // columns held in registers across the epilogues spilled)
                        const bool okc = jj4[r] < A->n_up;
                        const int tcol = okc ? (int)c_up[okc ? jj4[r] : 0] : D;
                        xt[(16 * s + sl) * XS + tcol] = out;
                        ldsum[s] += (inside && live) ? lad : 0.0f;
                        any_in |= inside && live;
                        any_nd |= nd && inside && live;
                    }
                }
            }
            epi_end();
        }
        // end of the layer: log|det| in the order of per-layer launches, status bits
#pragma unroll
        for (int s = 0; s < NTL; ++s) {
            float v = ldsum[s];
            v += __shfl_xor(v, 16, 64);
            v += __shfl_xor(v, 32, 64);
            ld_acc[s] = ld_acc[s] + v;
        }
        const int bits = (__any(any_in) ? NFK_ST_INSIDE_SEEN : 0) | (__any(any_nd) ? NFK_ST_NEG_DISC : 0);
        if (lane == 0 && bits != 0) atomicOr(cst + l, bits);
    }

    // ---- tail: z rows (or the prior epilogue), log|det|, status words
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int D4 = D >> 2;
    if (A->z != nullptr)
        for (RowWalk w(lane, D4); w.r < nall; w.next()) {
            const float* row = xt + w.r * XS;
            const int o = 4 * w.k;
            *reinterpret_cast<float4*>(A->z + (b0 + w.r) * A->ldz + o) =
                make_float4(row[c_src[o]], row[c_src[o + 1]], row[c_src[o + 2]], row[c_src[o + 3]]);
        }
#pragma unroll
    for (int s = 0; s < NTL; ++s) {
        if (q == 0 && row_ok[s] && A->mode != 0) A->logdet[b0 + 16 * s + sl] = ld_acc[s];
        if (A->log_prob != nullptr) {
            const float* row = xt + (16 * s + sl) * XS;
            const float il = A->prior_inv_scale;
            float m = 0.0f;
            for (int g = q; g < D4; g += 4) {
                const int o = 4 * g;
                const float y0 = row[c_src[o]] * il, y1 = row[c_src[o + 1]] * il;
                const float y2 = row[c_src[o + 2]] * il, y3 = row[c_src[o + 3]] * il;
                m += (y0 * y0 + y1 * y1) + (y2 * y2 + y3 * y3);
            }
            m += __shfl_xor(m, 16, 64);
            m += __shfl_xor(m, 32, 64);
            const float lp = -0.5f * (A->prior_c2pi + m) - A->prior_hld;
            if (q == 0 && row_ok[s]) A->log_prob[b0 + 16 * s + sl] = lp + ld_acc[s];
            if (__any(row_ok[s] && m != m) && lane == 0) atomicOr(cst, NFK_ST_NAN_Z);
        }
    }
    __syncthreads();
    if (A->status != nullptr && (int)threadIdx.x < NL) {
        const int bits = cst[threadIdx.x];
        if (bits != 0 && (A->status[threadIdx.x] & bits) != bits) atomicOr(A->status + threadIdx.x, bits);
    }
}

// c3-class instances of the two-tile chain: (KBH, T1, K)
#define NFK_CHAIN2_SHAPES(X) X(3, 1, 8)

int launch_chain2(const FusedArgs& a, const Layout& L, int K, bool inv, hipStream_t st) {
    const int64_t per = (int64_t)kNsfWaves * 16 * kC2Tiles;
    const int64_t blocks = (a.batch + per - 1) / per;
    if (blocks == 0) return 0;
    const size_t lds = lds_bytes_chain2(L, a.nlayers, a.saves != nullptr);
    const dim3 g((unsigned)blocks), b(64 * kNsfWaves);
#define NFK_C2(h, t, k)                                                                  \
    if (L.KBH == h && L.T1 == t && K == k) {                                             \
        if (inv)                                                                         \
            hipLaunchKernelGGL((k_nsf_chain2<h, t != 0, k, true>), g, b, lds, st, a);    \
        else                                                                             \
            hipLaunchKernelGGL((k_nsf_chain2<h, t != 0, k, false>), g, b, lds, st, a);   \
        hipError_t e = hipGetLastError();                                                \
        return e == hipSuccess ? 0 : (int)e;                                             \
    }
    NFK_CHAIN2_SHAPES(NFK_C2)
#undef NFK_C2
    return -1;  // no instance
}

bool chain2_ok(const Layout& L, int K, int nl, bool saved) {
    bool inst = false;
#define NFK_C2CHK(h, t, k) inst |= (L.KBH == h && L.T1 == t && K == k);
    NFK_CHAIN2_SHAPES(NFK_C2CHK)
#undef NFK_C2CHK
    return inst && L.n_lo <= 32 && 2 * lds_alloc(lds_bytes_chain2(L, nl, saved)) <= (size_t)kLdsBytes &&
           (!saved || (L.n_lo + L.n_up) % 4 == 0);
}

}  // namespace nfk_fused
