// nfk_fused_impl.h -- fused NSF coupling-layer kernel; design notes in nfk_fused.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "../../include/nfk.h"
#include "nfk_spline.h"

int nfk_set_error(const char* msg);  // nfk_kernels.hip

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

#ifndef NFK_WAVES
#define NFK_WAVES 8
#endif
#ifndef NFK_NSF_WAVES
#define NFK_NSF_WAVES 4  // waves per workgroup of k_fused_nsf (one per SIMD)
#endif
#ifndef NFK_SPLIT_NS
#define NFK_SPLIT_NS 4  // split form: tiles per sub-record (KBH <= 3)
#endif
#ifndef NFK_NSF_WPE_SPLIT
#define NFK_NSF_WPE_SPLIT 3  // split form: workgroups per CU (waves per SIMD)
#endif
#ifndef NFK_GEMM_PF
#define NFK_GEMM_PF 1  // gemm_h: prefetch the next tile pair's A fragments (register ring)
#endif
#ifndef NFK_SPLIT_PIPE
#define NFK_SPLIT_PIPE 1  // split form: pipelined chunk schedule where it applies
#endif
#ifndef NFK_LDS_PAD
#define NFK_LDS_PAD 0  // diagnostic: extra LDS per k_fused_nsf workgroup (fewer per CU)
#endif

namespace nfk_fused {

constexpr int kWaves = NFK_WAVES;  // waves per workgroup (two per SIMD by default), 16 samples each
constexpr int kNsfWaves = NFK_NSF_WAVES;
constexpr int kMaxD = 128;
constexpr int kLdsBytes = 160 * 1024;
constexpr float kActScale = 16384.0f;  // tanh outputs are split at 2^14 (|h| * 2^14 <= 2^14)

// ---------------------------------------------------------------------------
// Packed weights ("pack"): a header block, then a stream of phase records.
// A record is a run of 1-KiB blocks (64 lanes x 16 B, one wave-instruction of
// global_load_lds each) followed by one bias block (float[16 tiles][16 rows]).
//   header (1 block): hdr[0..2] = max|W1|, max|W2|, max|W3| (uint bits, from
//            the pack's reduction); float hdr[3] = 2^-s1, hdr[4] = 2^-(s2+14),
//            hdr[5] = 2^-(s3+14): the factors undoing the fp16 pre-scaling
//   f16 blocks (v_mfma_f32_16x16x32_f16, two-way split): k-blocks x NT tiles
//            x {hi, lo}: lane l of block (kb, t, p) holds part p of
//            2^s W[row(t, l&15)][32kb + 8(l>>4) + j], j = 0..7, where hi = f16(v),
//            lo = f16(v - hi) and 2^s puts max|W| in [2^14, 2^15)
//   tail (T1 only: H = 32 KBH + R, 0 < R <= 4, one v_mfma_f32_16x16x16_f16
//            per tile): one block per 2 tiles; lane l's 16 B hold tile 2g's
//            then tile 2g + 1's fragment, 4 halves over the tail features
//            32 KBH + 0..3 of row(t, l&15): k-group l>>4 = {hi, hi, lo, 0} of 2^s W, against
//            the B groups {a_hi, a_lo, a_hi, -} (tail_word, act_operands): the
//            same three split products as the k-blocks, in one f16 MFMA
//   layer 1: KB1 = ceil(n_lo/32) f16 k-blocks (x is scaled per sample, by a power of two), bias unscaled
//   layer 2: KBH f16 k-blocks (+ tail blocks), bias pre-scaled by 2^(s2+14)
//   per 16-coordinate chunk: W logits (K tiles), H logits (K tiles), D logits
//            (K-1 tiles), same form; row i of tile t = parameter t of coordinate 16c+i
// Hidden feature permutation: row i of hidden tile t < 2 KBH computes feature
//   f(t, i) = 32(t>>1) + 8(i>>2) + 4(t&1) + (i&3),
// so accumulator register r of tiles 2kb, 2kb+1 of lane l are exactly
// elements j = r, 4 + r of the next product's B fragment for k-block kb
// (k = 32kb + 8(l>>4) + j) -- activations never leave registers.  With a
// tail, tile 2 KBH holds features 32 KBH + r in register r of every lane
// group (rows duplicated): the B operand of the tail step needs all R in
// each lane.
// wide = 1 (nfk_fused_wide.h): the output layer in 8-coordinate chunks whose
//   W/H/D records have ceil(K/2) tiles; row i of tile t = parameter
//   2t + (i&1) of coordinate 8c + 2(i>>2) + ((i>>1)&1), so lane group q holds
//   two coordinates with all their parameters in registers 2h, 2h+1 of the
//   tiles (half the accumulators of the 16-coordinate form).
// Diagnostic timeline (-DNFK_TRACE builds only, tools/trace_wide.py): each
// wave records s_memtime at marked points into lanes of 4 VGPRs (256 marks);
// every 512th workgroup writes them to a buffer set by nfk_debug_trace().
struct NfkTrace {
    uint32_t v0 = 0, v1 = 0, v2 = 0, v3 = 0;
    int n = 0;
};
#ifdef NFK_TRACE
__device__ __forceinline__ void nfk_mark(NfkTrace& t) {
    const uint32_t c = (uint32_t)__builtin_readcyclecounter();
    const int i = t.n & 255;
    const bool me = (int)(threadIdx.x & 63) == (i & 63);
    if (t.n > 255) return;  // first 256 marks only (persistent kernels: the first tiles)
    if (i < 64)
        t.v0 = me ? c : t.v0;
    else if (i < 128)
        t.v1 = me ? c : t.v1;
    else if (i < 192)
        t.v2 = me ? c : t.v2;
    else
        t.v3 = me ? c : t.v3;
    ++t.n;
}
__device__ __forceinline__ void nfk_trace_flush(const NfkTrace& t, uint32_t* buf, int wid, int lane) {
    if (buf == nullptr || (blockIdx.x & 511) != 0) return;
    uint32_t* o = buf + ((size_t)(blockIdx.x >> 9) * 16 + wid) * 260;
    o[lane] = t.v0;
    o[64 + lane] = t.v1;
    o[128 + lane] = t.v2;
    o[192 + lane] = t.v3;
    if (lane == 0) o[256] = (uint32_t)t.n;
}
#define NFK_MARK(t) nfk_mark(t)
#else
#define NFK_MARK(t) ((void)0)
#endif

struct Layout {
    int n_lo, n_up, H, K, P, KBH, T1, HT, KB1, NCH, wide, CW;
    int blk_h1, blk_h2, blk_w, blk_d, blk_chunk, slot_blocks;
    int64_t o_h1, o_h2, o_w3, total;  // offsets / size in floats
};

// blocks of an f16-split record with nt tiles (+ tail blocks, + bias)
inline int rec_blocks(int kbh, int t1, int nt) { return kbh * nt * 2 + (t1 ? (nt + 1) / 2 : 0) + 1; }

inline Layout make_layout(int n_lo, int n_up, int H, int K, int wide = 0) {
    Layout L;
    L.wide = wide;
    L.CW = wide ? 8 : 16;
    L.n_lo = n_lo;
    L.n_up = n_up;
    L.H = H;
    L.K = K;
    L.P = 3 * K - 1;
    const int kbf = H / 32, rem = H - 32 * kbf;
    if (rem == 0) {
        L.KBH = kbf;
        L.T1 = 0;
    } else if (rem <= 4 && kbf >= 1) {
        L.KBH = kbf;
        L.T1 = 1;
    } else {
        L.KBH = kbf + 1;
        L.T1 = 0;
    }
    L.HT = 2 * L.KBH + L.T1;
    L.KB1 = (n_lo + 31) / 32;
    L.NCH = (n_up + L.CW - 1) / L.CW;
    L.blk_h1 = L.KB1 * L.HT * 2 + 1;
    L.blk_h2 = rec_blocks(L.KBH, L.T1, L.HT);
    L.blk_w = rec_blocks(L.KBH, L.T1, wide ? (K + 1) / 2 : K);
    L.blk_d = rec_blocks(L.KBH, L.T1, wide ? K / 2 : K - 1);
    L.blk_chunk = 2 * L.blk_w + L.blk_d;
    L.slot_blocks = L.blk_h1;
    if (L.blk_h2 > L.slot_blocks) L.slot_blocks = L.blk_h2;
    if (L.blk_w > L.slot_blocks) L.slot_blocks = L.blk_w;
    if (L.blk_d > L.slot_blocks) L.slot_blocks = L.blk_d;
    L.o_h1 = 256;  // after the header block
    L.o_h2 = L.o_h1 + (int64_t)L.blk_h1 * 256;
    L.o_w3 = L.o_h2 + (int64_t)L.blk_h2 * 256;
    L.total = L.o_w3 + (int64_t)L.NCH * L.blk_chunk * 256;
    return L;
}

// Each wave owns two x tiles, filled in the prologue by per-lane LDS-DMA
// gathers of 64 dwords: 16 rows of the lower coordinates (padded to the
// layer-1 k-blocks) and 16 rows of the upper ones (padded to 4).  The upper
// tile also collects the transformed values, so z is written once at the end.
inline int x_lo_row(const Layout& L) { return 32 * L.KB1; }
inline int x_up_row(const Layout& L) { return (L.n_up + 3) & ~3; }
inline int x_tile_floats(const Layout& L) { return 16 * (x_lo_row(L) + x_up_row(L)); }

// dynamic LDS bytes of k_fused_nsf: the record slot, the index maps, the x
// tiles of every wave
inline size_t lds_bytes(const Layout& L) {
    const int D = L.n_lo + L.n_up;
    const size_t maps = (size_t)((2 * D + 3) / 4) * 16;
    return (size_t)L.slot_blocks * 1024 + maps + (size_t)kNsfWaves * x_tile_floats(L) * sizeof(float) +
           (size_t)kNsfWaves * L.K * 64 * sizeof(int) +  // bin lookup tables
           NFK_LDS_PAD;
}

// Split form (NfkSplit): slot of KBH NS 2 + T1 NS/2 + 1 blocks (at least the
// layer-1 record); used when three workgroups then fit a CU.
inline int split_slot_blocks(const Layout& L) {
    const int ns = L.KBH <= 3 ? NFK_SPLIT_NS : 2;
    const int sb = L.KBH * ns * 2 + (L.T1 ? (ns + 1) / 2 : 0) + 1;
    return sb > L.blk_h1 ? sb : L.blk_h1;
}
// split-form LDS: the slot, four maps + the output->input column map, each
// wave's [16][D + 1] tile of whole x rows, the lookup tables
inline size_t lds_bytes_split(const Layout& L) {
    const int D = L.n_lo + L.n_up;
    return (size_t)split_slot_blocks(L) * 1024 + (size_t)((3 * D + 3) / 4) * 16 +
           (size_t)kNsfWaves * 16 * (D + 1) * sizeof(float) + (size_t)kNsfWaves * L.K * 64 * sizeof(int) +
           NFK_LDS_PAD;
}
// chain form: the maps region holds (nl + 1) D ints instead of 3 D
inline size_t lds_bytes_chain(const Layout& L, int nl) {
    const int D = L.n_lo + L.n_up;
    return lds_bytes_split(L) - (size_t)((3 * D + 3) / 4) * 16 + (size_t)((4 * nl + (nl + 1) * D + 15) / 16) * 16;
}
// shape conditions of the split form (the launch also needs 16-B aligned x
// and z rows: D, ldx, ldz multiples of 4)
inline bool split_ok(const Layout& L) {
    return L.wide == 0 && (L.n_lo + L.n_up) % 4 == 0 && NFK_NSF_WPE_SPLIT * lds_bytes_split(L) <= (size_t)kLdsBytes;
}

// most layers one chain launch may hold with three workgroups per CU (status
// bits ride one lane per layer: at most 64); 0 if the split form does not apply
// (with LDS counted in 1280-byte allocation units, the coarsest granule
// measured: a chain 32 B over a third of the CU's LDS lost its third
// workgroup).  Map bytes limit D to 128 (kMaxD).
constexpr size_t kLdsGranule = 1280;
inline size_t lds_alloc(size_t b) { return (b + kLdsGranule - 1) / kLdsGranule * kLdsGranule; }
inline int chain_max_layers(const Layout& L) {
    if (!split_ok(L) || L.n_lo + L.n_up > 128) return 0;
    int n = 0;
    while (n < 64 && NFK_NSF_WPE_SPLIT * lds_alloc(lds_bytes_chain(L, n + 1)) <= (size_t)kLdsBytes) ++n;
    return n;
}

// hidden feature computed by row i (0..15) of hidden tile t (>= H: padding)
__host__ __device__ inline int hid_feature(int t, int i, int kbh) {
    if (t < 2 * kbh) return 32 * (t >> 1) + 8 * (i >> 2) + 4 * (t & 1) + (i & 3);
    return 32 * kbh + (i & 3);  // the tail tile: every lane group holds the tail features
}

// f16 pair (v0, v1) of split part p (0 = hi, 1 = lo) as one packed word
__device__ __forceinline__ uint32_t nfk_f16_part_pair(float v0, float v1, int part) {
    const _Float16 h0 = (_Float16)v0, h1 = (_Float16)v1;
    const _Float16 r0 = part ? (_Float16)(v0 - (float)h0) : h0;
    const _Float16 r1 = part ? (_Float16)(v1 - (float)h1) : h1;
    return (uint32_t)__builtin_bit_cast(uint16_t, r0) | ((uint32_t)__builtin_bit_cast(uint16_t, r1) << 16);
}

// Word wl (0..255) of tail block g of a record with nt tiles (the 16x16x16 f16
// A fragments of tiles 2g and 2g + 1, interleaved per lane: words 4l, 4l + 1
// tile 2g, 4l + 2, 4l + 3 tile 2g + 1): lane l of tile t holds halves j = 0..3 =
// tail features kbase + j of weight row row_of(t, l & 15), as the hi part in
// k-groups 0 and 1, the lo part in k-group 2, zero in k-group 3.
template <class RowF>
__device__ uint32_t tail_word(int g, int wl, int nt, int kbase, int H, float sc, RowF row_of) {
    const int t = 2 * g + ((wl & 3) >> 1), lane = wl >> 2, j = 2 * (wl & 1), q = lane >> 4;
    if (t >= nt || q == 3) return 0u;
    const float* w = row_of(t, lane & 15);
    float v0 = 0.0f, v1 = 0.0f;
    if (w != nullptr) {
        if (kbase + j < H) v0 = w[kbase + j] * sc;
        if (kbase + j + 1 < H) v1 = w[kbase + j + 1] * sc;
    }
    return nfk_f16_part_pair(v0, v1, q == 2 ? 1 : 0);
}

// Spline constants of NSF_CL (flows.py:236: left = bottom = -B, right = top = B,
// default min bin width = height = derivative = 1e-3), one set for x and y.
struct FusedConst {
    float lo, hi;     // -B, B (knot range and the tails' inside test)
    float sp30;       // 2B * 2^-30: fixed-point prefix -> edge offset
    float inv30;      // 2^30 / 2B: x -> fixed-point domain
    float fb30, mb30; // (1 - min_bin K) 2^30, min_bin 2^30: floored fractions in fixed point
    float m2b;        // 2B log2(e): second softmax (nfk_knots_nsf_lean)
    float min_d;      // min_derivative
    float d_edge;     // min_d + softplus(pad constant): boundary derivative
};

struct FusedArgs {
    const float* x;
    const float* pack;
    const int32_t *up_in, *up_out, *lo_in, *lo_out;
    float* z;
    float* logdet;
    int32_t* status;
    int64_t ldx, ldz, batch;
    int32_t n_lo, n_up, KB1, NCH, mode, slot_blocks, xtile, xup;
    int32_t blk_h1, blk_h2, blk_w, blk_d, blk_chunk;
    int32_t o_h1, o_h2, o_w3;  // float offsets into pack (< 2^31 by shape limits)
    FusedConst c;
    uint32_t* trace;  // diagnostic timeline buffer (NFK_TRACE builds), else unused
    // chain form (k_fused_nsf<..., CHAIN = true>): nlayers layers of one shape in
    // one launch, x rows resident in the LDS tile from the first layer to the last
    const float* const* packs;  // device array: the packs of the layers, in execution order
    const int32_t* cmaps;       // [nlayers][n_lo + n_up] tile columns (lower, then upper)
                                // of every layer's inputs, then [D] the tile column of
                                // every output column after the last layer
    int32_t nlayers;
    // chain form, optional prior epilogue: log_prob[b] = log N(z_b; 0, s^2 I) +
    // log|det|_b (z need not be written then: z may be null)
    float* log_prob;
    float prior_inv_scale, prior_c2pi, prior_hld;
    // two-tile chain, training form (nfk_fused_nsf_chain_saved): the input of
    // every layer l >= 1 written to saves + (l - 1) save_stride (rows of
    // ld_saves floats) through smaps [(nlayers - 1) D] (tile column of each of
    // that layer's input columns); saves null otherwise
    float* saves;
    int64_t ld_saves, save_stride;
    const int32_t* smaps;
};

__device__ __forceinline__ f32x4 mfma16(h8 a, h8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// the tail step: K = 16 over the packed (hi, hi, lo, 0) x (a_hi, a_lo, a_hi, -) groups
__device__ __forceinline__ f32x4 mfma16k16(h4 a, h4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 as_f32x4(const float4& v) {
    f32x4 r;
    r[0] = v.x;
    r[1] = v.y;
    r[2] = v.z;
    r[3] = v.w;
    return r;
}

// LDS-DMA is issued through inline asm and waited for by hand: the compiler
// cannot prove that a DMA into one slot does not alias reads of the other, so
// with the builtin it drains every DMA (vmcnt(0)) before the first ds_read of
// each phase -- serialising the copy of phase p+1 with the compute of phase p.
// Invariant instead: a DMA issued right after the barrier that ends phase p
// is waited for (vmcnt(0)) at the barrier that ends phase p+1, and the kernel
// issues no other VGPR-destination global loads while DMAs are in flight.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

__device__ __forceinline__ void dma16(const float* gsrc, uint32_t lds) {
    uint32_t saved;  // m0 is reserved by the compiler: restore it
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(saved)
                 : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(gsrc)
                 : "memory");
}

// The same from a WAVE-UNIFORM source address: the saddr form (SGPR base +
// a 32-bit per-lane VGPR offset), so stepping the source costs two SALU adds
// instead of a 64-bit VALU add per lane and block.  Off by default: measured
// 3 % SLOWER on the c3 chain (5.57 vs 5.39-5.42 ms per launch, A/B on one box,
// profiles/r4v_c3_variants.txt) -- the v_readfirstlane of a VGPR-computed
// base puts a VALU -> SALU dependency in front of every copy
#ifndef NFK_DMA_SADDR
#define NFK_DMA_SADDR 0
#endif
__device__ __forceinline__ void dma16u(const float* gbase, uint32_t voff, uint32_t lds) {
    const uint64_t p = (uint64_t)gbase;
    // (readfirstlane returns int: each half through uint32_t, or the low half
    // would sign-extend into the high one)
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)p);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32));
    const uint64_t ps = ((uint64_t)hi << 32) | (uint64_t)lo;
    uint32_t saved;  // m0 is reserved by the compiler: restore it
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %2, %3\n\ts_mov_b32 m0, %0"
                 : "=&s"(saved)
                 : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(voff), "s"(ps)
                 : "memory");
}
// one 1-KiB block at uniform address g (lane l copies bytes 16 l .. 16 l + 15)
__device__ __forceinline__ void dma_blk(const float* g, int lane, uint32_t lds) {
#if NFK_DMA_SADDR
    dma16u(g, (uint32_t)lane * 16u, lds);
#else
    dma16(g + lane * 4, lds);
#endif
}

__device__ __forceinline__ void dma4(const float* gsrc, uint32_t lds) {
    uint32_t saved;  // m0 is reserved by the compiler: restore it
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "global_load_lds_dword %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(saved)
                 : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(gsrc)
                 : "memory");
}

// dma4 with the non-temporal cache policy: for bytes one workgroup reads once
// (x rows), so they do not displace the weight records every workgroup re-reads.
// NFK_X_NT: the chains' x rows (c3, c2) by this policy -- HBM traffic per launch
// 1.27x -> 1.09x of the algorithmic bytes at c3, 1.14x -> 1.09x at c2, time
// within 0.3 % (profiles/r5/r5zc_c3_x_nt_ab.txt, r5zd_c2_x_nt_ab.txt)
#ifndef NFK_X_NT
#define NFK_X_NT 1
#endif
__device__ __forceinline__ void dma4_nt(const float* gsrc, uint32_t lds) {
    uint32_t saved;  // m0 is reserved by the compiler: restore it
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
                 "global_load_lds_dword %2, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(saved)
                 : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(gsrc)
                 : "memory");
}

// every DMA and LDS access of this wave retired, then the workgroup barrier
// Kernels that issue MFMAs and can share a SIMD with other waves are
// code-generated without packed-FP32 VALU instructions (v_pk_{add,mul,fma}_f32):
// DESIGN.md section 10.5 -- with dependent MFMA accumulate chains in flight on
// the SIMD, packed-FP32 results in lanes 48-63 of a co-resident wave were
// intermittently wrong (tools/ubench_elem_twice.hip reproduces it; the same
// source without packed FP32 never does).  The MFMA translation units are built
// without the feature (Makefile NOPK); a kernel that runs one wave per SIMD
// (512 registers) may take it back with NFK_PK_FP32.  (The other way round --
// a per-kernel "no-packed-fp32-ops" in a packed unit -- stops the inliner:
// lambdas keep the unit's features and became calls.)
#if defined(__HIP_DEVICE_COMPILE__)
#define NFK_PK_FP32 __attribute__((target("packed-fp32-ops")))
#else
#define NFK_PK_FP32  // (a device feature: the host pass does not know it)
#endif

// s_waitcnt vmcnt(n) for a wave-uniform n known only at run time (the field is
// an immediate): a branch to the matching wait; n >= 63 waits for 63
__device__ __forceinline__ void wait_vmcnt_le(int n) {
    n = __builtin_amdgcn_readfirstlane(n);
    switch (n < 63 ? n : 63) {
#define NFK_VMW(k) \
    case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
#define NFK_VMW8(k) NFK_VMW(k) NFK_VMW(k + 1) NFK_VMW(k + 2) NFK_VMW(k + 3) NFK_VMW(k + 4) NFK_VMW(k + 5) \
    NFK_VMW(k + 6) NFK_VMW(k + 7)
        NFK_VMW8(0) NFK_VMW8(8) NFK_VMW8(16) NFK_VMW8(24) NFK_VMW8(32) NFK_VMW8(40) NFK_VMW8(48)
        NFK_VMW(56) NFK_VMW(57) NFK_VMW(58) NFK_VMW(59) NFK_VMW(60) NFK_VMW(61) NFK_VMW(62)
        default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
#undef NFK_VMW8
#undef NFK_VMW
    }
}

__device__ __forceinline__ void dma_barrier() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// Copy one phase record (nblk 1-KiB blocks at src) into an LDS slot: block i
// goes by wave i % NW as one global_load_lds_dwordx4 (LDS destination =
// wave-uniform base + 16 B x lane).
template <int NW = kWaves>
__device__ __forceinline__ void stage_record(const float* __restrict__ src, int nblk, float4* slot,
                                             int wid, int lane) {
    const uint32_t base = lds_addr(slot);
    for (int i = wid; i < nblk; i += NW) dma_blk(src + (int64_t)i * 256, lane, base + i * 1024);
}

// Walk the elements e = lane, lane + 64, ... of a [rows][row] tile as
// (r, k) = (e / row, e % row) with one division up front (the loops below ran
// a VALU integer division per element).
struct RowWalk {
    int r, k, dr, dk, row;
    __device__ __forceinline__ RowWalk(int lane, int row_) : row(row_) {
        r = lane / row;
        k = lane - r * row;
        dr = 64 / row;
        dk = 64 - dr * row;
    }
    __device__ __forceinline__ void next() {
        k += dk;
        r += dr;
        if (k >= row) {
            k -= row;
            ++r;
        }
    }
};

// Gather a [16][row] tile of x (rows b0.., columns map[0..n)) into this wave's
// LDS tile: element e = 64 i + lane of instruction i is (e / row, e % row).
// Padding columns and rows past the batch re-read a valid element (their
// weights are zero / their results are dropped).
__device__ __forceinline__ void gather_x(const float* __restrict__ x, int64_t ldx, int64_t b0, int nrows,
                                         const int32_t* map, int n, int row, float* tile, int lane) {
    const uint32_t base = lds_addr(tile);
    RowWalk w(lane, row);
    for (int i = 0; i < row / 4; ++i, w.next()) {
        const int64_t rr = b0 + (w.r < nrows ? w.r : 0);
        dma4(x + rr * ldx + map[w.k < n ? w.k : 0], base + i * 256);
    }
}

// tanh of acc * unscale, returned times 2^14 (ready for the fp16 split):
// sign(x) (1 - t) / (1 + t), t = 2^(-2|x| log2e) in (0, 1]; c2 = -2 log2e
// unscale.  Branch free, no overflow; absolute error ~1e-7 of the activation
// (which only feeds the next linear layer, where absolute error propagates).
// NFK_TANH6: 1 (default) 2^14 tanh = 2^15 / (1 + t) - 2^14 on t = e^(-2|x|), 6 VALU;
// 0 the rounds 1-4 form (1 - t) / ((1 + t) / 2^14), 7 VALU; 2 a 5-VALU signed form.
// A/B on one box (profiles/r5/r5s_tanh_ab.txt, kernel means of 3 runs): c2 chain
// 4.849 / 4.702 / 4.768 ms, c3 chain 5.407 / 5.370 / 5.405 ms, Gaussian NSF_AR
// 6.16 / - / 6.01 ms for 0 / 1 / 2; parity vs the oracle unchanged (7.6e-7 max rel.)
#ifndef NFK_TANH6
#define NFK_TANH6 1
#endif
#ifndef NFK_SPLIT_MIX
#define NFK_SPLIT_MIX 1
#endif
__device__ __forceinline__ float tanh_scaled(float acc, float c2) {
#if NFK_TANH6 == 2
    // (A/B) 2^14 tanh(x) = 2^14 - 2^15 / (1 + e^(2x)) on the signed x: e^(2x)
    // overflows to +inf for large x (the quotient to 0, tanh to 1) and
    // underflows to 0 for large -x (tanh -1), so neither |x| nor copysign is
    // needed: 5 VALU (mul, exp, add, rcp, fma)
    const float t = __builtin_amdgcn_exp2f(acc * -c2);
    return __builtin_fmaf(-2.0f * kActScale, __builtin_amdgcn_rcpf(1.0f + t), kActScale);
#else
    const float t = __builtin_amdgcn_exp2f(__builtin_fabsf(acc) * c2);
#if NFK_TANH6  // (A/B) 2^14 tanh = 2^15 / (1 + t) - 2^14: one VALU fewer
    const float r = __builtin_fmaf(2.0f * kActScale, __builtin_amdgcn_rcpf(1.0f + t), -kActScale);
#else
    const float inv = 1.0f / kActScale;
    const float r = (1.0f - t) * __builtin_amdgcn_rcpf(__builtin_fmaf(t, inv, inv));
#endif
    return __builtin_copysignf(r, acc);
#endif
}

// the fp16 residuals of (v0, v1) over their fp16 roundings (the halves of
// hp): v - h is exact in fp32, so fma(h, -1, v) rounded once to fp16 is
// bitwise (_Float16)(v - (float)h).  As an fma of an fp16 and an fp32 operand
// with an fp16 result, written into either half of the packed pair, that is
// ONE v_fma_mix{lo,hi}_f16 per element instead of an fp16 -> fp32 convert, a
// subtract and an fp32 -> fp16 convert (hipcc turns fma(h, -1, v) back into the
// subtract, hence the asm).  NFK_SPLIT_MIX=0: the plain expression.
__device__ __forceinline__ uint32_t f16_residual_pair(float v0, float v1, uint32_t hp) {
#if NFK_SPLIT_MIX
    uint32_t r;
    asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(hp), "v"(v0));
    asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(r) : "v"(hp), "v"(v1));
    return r;
#else
    const _Float16 h0 = __builtin_bit_cast(_Float16, (uint16_t)(hp & 0xFFFFu));
    const _Float16 h1 = __builtin_bit_cast(_Float16, (uint16_t)(hp >> 16));
    const _Float16 l0 = (_Float16)(v0 - (float)h0), l1 = (_Float16)(v1 - (float)h1);
    return (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
#endif
}

// B fragments (hi, lo) of k-block kb from the activations of tiles 2kb, 2kb+1
template <int HT>
__device__ __forceinline__ void split_act(const f32x4 (&a)[HT], int kb, h8& hi, h8& lo) {
#pragma unroll
    for (int j = 0; j < 8; ++j) hi[j] = (_Float16)a[2 * kb + (j >> 2)][j & 3];
#if NFK_SPLIT_MIX
    const u32x4 hp = __builtin_bit_cast(u32x4, hi);
    u32x4 lp;
#pragma unroll
    for (int p = 0; p < 4; ++p)
        lp[p] = f16_residual_pair(a[2 * kb + (p >> 1)][2 * (p & 1)], a[2 * kb + (p >> 1)][2 * (p & 1) + 1], hp[p]);
    lo = __builtin_bit_cast(h8, lp);
#else
#pragma unroll
    for (int j = 0; j < 8; ++j) lo[j] = (_Float16)(a[2 * kb + (j >> 2)][j & 3] - (float)hi[j]);
#endif
}

// Wait after a GEMM's last MFMA before its accumulators are read (32 wait
// states).  Measured on the wide fused NSF_AR (nfk_fused_ar.hip, one wave per
// SIMD, accumulators in AGPRs): without it the last output tile's register 3
// (the MFMA's last-written rows) was read stale in some builds -- the compiler's
// own MFMA -> read wait states did not cover it (tools/dbg_ar_dump.py,
// profiles/r4_ar_wide_debug.txt).
// Fence that ends a GEMM segment before its workgroup barrier.  The barrier
// and the copy waits are inline asm, which orders memory operations only: the
// compiler sank a segment's last MFMAs below the barrier, and on the path that
// skips the next copy (the stream's last sub-records) the allocator's AGPR ->
// VGPR copies of their accumulators followed ~3 instructions after the MFMA --
// stale rows on gfx950 (tools/ubench_mfma_raw.hip: a v_accvgpr_read of a
// 16x16x32 MFMA result needs 5-8 wait states; profiles/r4_mfma_hazards.txt).
// The scheduling fence keeps every MFMA above the barrier and the s_nop gives
// the last one its wait states.
__device__ __forceinline__ void gemm_fence() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7");
    __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void mfma_result_wait() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7");
    __builtin_amdgcn_sched_barrier(0);
}

// acc[t] = bias + 2^s W[tile t] . act^T: KBH k-blocks of 32 in the fp16
// split, three MFMAs per (tile, k-block), small terms first, then the tail
// step (T1: one f16 MFMA holding the three split products of the <= 4 tail
// features, its fragments carried by the same prefetch ring).
// Tiles go in pairs whose MFMAs alternate accumulators: a dependent MFMA
// chain blocks the SIMD partner wave's VALU, two interleaved chains let it
// overlap (tools/ubench_coexec2.hip, modes 5-6).  A fragments of the next
// pair are read from the LDS slot while the current pair's MFMAs run.
// Split form (sub-records, k_fused_nsf<..., SPLIT = true>): the slot holds
// tiles [T0, T0 + NT) of a record, at a tile stride of NS per k-block, then
// the tail blocks holding them and the record's whole bias block; acc has NA
// tiles and this call fills acc[T0 .. T0 + NT).  Whole records: NS = NA = NT.
// BREL: the sub-record's bias block holds its own tiles (row t - T0; records
// of more than 16 tiles, whose biases exceed one 1-KiB block); else the
// record's whole bias block (tile t at row t).
// WAIT: the last MFMA's results are read soon after (a record's last
// sub-record): wait them out here (see kMfmaResultWait).
template <int KBH, bool T1, int NT, int NS = NT, int T0 = 0, int NA = NT, bool BREL = false, bool WAIT = false>
__device__ __forceinline__ void gemm_h(const h8 (&bh)[KBH], const h8 (&bl)[KBH], h4 btail,
                                       const float4* slot, int lane, f32x4 (&acc)[NA], float bsc = 1.0f) {
    constexpr int NPR = (NT + 1) / 2;  // tile pairs (the last may be a single tile)
    constexpr int N = KBH * NPR;       // k-block steps; T1: then NPR tail steps
    constexpr int NI = N + (T1 ? NPR : 0);
    constexpr int NTG = T1 ? (NS + 1) / 2 : 0;
    const int q = lane >> 4;
    const float4* tail = slot + KBH * NS * 2 * 64;
    const float4* bias = tail + NTG * 64;
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[T0 + t] = as_f32x4(bias[((BREL ? 0 : T0) + t) * 4 + q]) * bsc;
#ifdef NFK_DIAG_BIAS_NOP  // diagnostic: a wait between the bias initialisation and the first MFMA
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#endif
    // fragments of step i into a ring slot: k-block step i = (kb, pr): tile
    // t0 = 2 pr {hi, lo}, tile t0 + 1 {hi, lo}; tail step N + pr: one 16-B
    // word per lane holding both tiles' tail fragments (tail block pr)
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
    if constexpr (NFK_GEMM_PF) fetch(0, ring[0]);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int pr = i < N ? i % NPR : i - N, kb = i < N ? i / NPR : 0, t0 = T0 + 2 * pr;
        const bool two = t0 + 1 < T0 + NT;
        if constexpr (!NFK_GEMM_PF)  // no prefetch: the step's fragments just before its MFMAs
            fetch(i, ring[i & 1]);
        else if (i + 1 < NI)
            fetch(i + 1, ring[(i + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        const float4* r = ring[i & 1];
        if (i >= N) {  // tail step (T1)
            if (i == N && NT <= 2) {
                // the tail MFMA (16x16x16) reads as its accumulator what a
                // 16x16x32 MFMA one or no instruction earlier wrote: across the
                // two opcodes the result is not forwarded (measured: rows 0, 1
                // of each lane group stale), so wait it out; with three or more
                // tiles two other MFMAs separate them
                __builtin_amdgcn_sched_barrier(0);
                if (NT == 1) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7");
                else asm volatile("s_nop 7\n\ts_nop 7");
#ifdef NFK_TAIL_NOP_EXTRA  // diagnostic: a longer wait before the tail step
                asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7");
#endif
                __builtin_amdgcn_sched_barrier(0);
            }
            const float4 w = r[0];
            acc[t0] = mfma16k16(__builtin_bit_cast(h4, make_float2(w.x, w.y)), btail, acc[t0]);
            if (two) acc[t0 + 1] = mfma16k16(__builtin_bit_cast(h4, make_float2(w.z, w.w)), btail, acc[t0 + 1]);
            continue;
        }
        const h8 ahi0 = __builtin_bit_cast(h8, r[0]), alo0 = __builtin_bit_cast(h8, r[1]);
#ifdef NFK_DIAG_MFMA_NOP  // diagnostic: a wait between the alternating MFMAs of a tile pair
#define NFK_MN() do { __builtin_amdgcn_sched_barrier(0); asm volatile("s_nop 7\n\ts_nop 3"); \
                      __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define NFK_MN() do { } while (0)
#endif
        if (two) {
            const h8 ahi1 = __builtin_bit_cast(h8, r[2]), alo1 = __builtin_bit_cast(h8, r[3]);
            acc[t0] = mfma16(alo0, bh[kb], acc[t0]);
            acc[t0 + 1] = mfma16(alo1, bh[kb], acc[t0 + 1]);
            NFK_MN();
            acc[t0] = mfma16(ahi0, bl[kb], acc[t0]);
            acc[t0 + 1] = mfma16(ahi1, bl[kb], acc[t0 + 1]);
            NFK_MN();
            acc[t0] = mfma16(ahi0, bh[kb], acc[t0]);
            acc[t0 + 1] = mfma16(ahi1, bh[kb], acc[t0 + 1]);
            NFK_MN();
        } else {
            acc[t0] = mfma16(alo0, bh[kb], acc[t0]);
            acc[t0] = mfma16(ahi0, bl[kb], acc[t0]);
            acc[t0] = mfma16(ahi0, bh[kb], acc[t0]);
        }
    }
    if constexpr (WAIT) mfma_result_wait();
}

// layer 1 from a whole layer-1 record (KBI f16 k-blocks x HT tiles, then the
// bias block): acc = b 2^(s1+sx) + 2^s1 W1 . (2^sx in)^T (fp16 split), the
// operands xh/xl of k-block kb holding inputs 32 kb + 8 q + j (in the
// record's input order)
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

// activations of a hidden layer -> B operands of the next product
// (T1: the tail B operand, k-groups {a_hi, a_lo, a_hi, a_hi} over the tail
// features held in registers 0..3 of the tail tile; A's group 3 is zero)
template <int KBH, bool T1, int HT>
__device__ __forceinline__ void act_operands(f32x4 (&h)[HT], float c2, h8 (&bh)[KBH], h8 (&bl)[KBH],
                                             h4& btail) {
#pragma unroll
    for (int t = 0; t < 2 * KBH; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) h[t][r] = tanh_scaled(h[t][r], c2);
#pragma unroll
    for (int kb = 0; kb < KBH; ++kb) split_act<HT>(h, kb, bh[kb], bl[kb]);
    if constexpr (T1) {
        h4 hi, lo;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float v = tanh_scaled(h[HT - 1][r], c2);
            h[HT - 1][r] = v;  // (kept like the other tiles' activations: store_act reads them)
            hi[r] = (_Float16)v;
            lo[r] = (_Float16)(v - (float)hi[r]);
        }
        btail = ((threadIdx.x >> 4) & 3) == 1 ? lo : hi;
    } else {
        btail = h4{0, 0, 0, 0};
    }
}

// Knot phase epilogue: for the 4 coordinates of this lane, turn the K logits
// of register r into fixed-point knot prefixes (NSF_CL's 2B softmax, then
// RQS's softmax, floor and cumsum: nfk_prefix_nsf_lean; the logits still carry
// the 2^(s3+14) product scale, which l2e absorbs) and keep (edge_k, size_k) of
// the bin.  The searched phase finds the bin in the integer domain:
// floor((x - lo) 2^30 / 2B) >= pre[j] counts the interior edges <= x, which is
// the bin of utils.py:20-25 for every x inside the tails (edges are strictly
// increasing; elements within an ulp of an edge may take the neighbouring
// bin, where the C1 spline agrees); the other phase selects by k.
// NFK_LUT (default): the two prefixes at the bin are read back from a per-wave
// LDS table (row j = prefix j of every lane, one ds_read2st64 at row k)
// instead of 2 (K-1) selects on compare masks.
#ifndef NFK_LUT
#define NFK_LUT 1
#endif
#ifndef NFK_E1_SEL
// knot_phase: the bin's right edge computed for every lane, then selected
#define NFK_E1_SEL 1
#endif
#ifndef NFK_PK2
// knot prefixes of coordinate pairs in packed fp32: 7 % fewer VALU
// instructions per layer, yet c3 measured 1 % slower (6.37 vs 6.30 ms per
// chain, A/B on one box), so off by default
#define NFK_PK2 0
#endif
template <int K, bool SEARCH, int R0 = 0, int R1 = 4, bool PK = true>
__device__ __forceinline__ void knot_phase(const f32x4 (&acc)[K], const float (&xv)[4],
                                           const FusedConst& c, float l2e, int (&kb)[4],
                                           float (&ek)[4], float (&sk)[4], int* scr, int lane) {
#ifdef NFK_ABL_NOEPI
#pragma unroll
    for (int r = R0; r < R1; ++r) {
        float v = 0.0f;
#pragma unroll
        for (int t = 0; t < K; ++t) v += acc[t][r];
        if (SEARCH) kb[r] = 0;
        ek[r] = v;
        sk[r] = xv[r];
    }
    return;
#endif
    // coordinate pairs (r, r + 1): the knot prefixes of both in packed fp32
    // (nfk_prefix_nsf_lean2, NFK_PK2; bitwise the per-coordinate result)
    constexpr bool PAIRS = PK && NFK_PK2 && K <= 8 && (R1 - R0) % 2 == 0;
    int pre2[K];
    float s2b = 0.0f;
#pragma unroll
    for (int r = R0; r < R1; ++r) {
        float u[K];
        int pre[K];
        float s2;  // the second softmax's sum: NaN iff a logit was NaN
#pragma unroll
        for (int t = 0; t < K; ++t) u[t] = acc[t][r];
        if constexpr (PAIRS) {
            if ((r - R0) % 2 == 0) {
                float u1[K];
#pragma unroll
                for (int t = 0; t < K; ++t) u1[t] = acc[t][r + 1];
                const nfk_f2 s = nfk_prefix_nsf_lean2<K>(u, u1, l2e, c.m2b, c.fb30, c.mb30, pre, pre2);
                s2 = s.x;
                s2b = s.y;
            } else {
#pragma unroll
                for (int t = 0; t < K; ++t) pre[t] = pre2[t];
                s2 = s2b;
            }
        } else {
            s2 = nfk_prefix_nsf_lean<K>(u, l2e, c.m2b, c.fb30, c.mb30, pre);
        }
        // the knot range's left end, NaN iff the logits were: the reference's NaN
        // cumsum makes every edge NaN (the integer prefixes would drop it)
        const float lo = __builtin_fmaf(s2, 0.0f, c.lo);
        int p0 = 0, p1 = pre[1 < K ? 1 : 0];
        if (SEARCH) {
            const int xi = __float2int_rd(__builtin_fmaf(xv[r], c.inv30, -c.lo * c.inv30));
            int k = 0;
#pragma unroll
            for (int j = 1; j < K; ++j) k += (xi >= pre[j]) ? 1 : 0;
            kb[r] = k;
        }
        const int kk = kb[r];
        if (NFK_LUT == 2 && SEARCH) {
            // (diagnostic A/B) the searched phase without the table: the
            // prefixes are strictly increasing from pre[0] = 0, so pre[kk] is
            // the largest prefix <= xi and pre[kk + 1] the smallest > xi, each
            // an unsigned minimum of differences (negative ones wrap high)
            const int xi = __float2int_rd(__builtin_fmaf(xv[r], c.inv30, -c.lo * c.inv30));
            uint32_t m0 = (uint32_t)xi, m1 = 0xffffffffu;
#pragma unroll
            for (int j = 1; j < K; ++j) {
                m0 = min(m0, (uint32_t)xi - (uint32_t)pre[j]);
                m1 = min(m1, (uint32_t)pre[j] - (uint32_t)xi - 1u);
            }
            p0 = (int)((uint32_t)xi - m0);
            p1 = (int)((uint32_t)xi + 1u + m1);
        } else if (NFK_LUT) {
            // rows 0..K-1; p1 is unused when kk = K - 1 (e1 = hi below)
#pragma unroll
            for (int j = 0; j < K; ++j) scr[j * 64 + lane] = pre[j];
            p0 = scr[kk * 64 + lane];
            p1 = scr[(kk + 1 < K ? kk + 1 : K - 1) * 64 + lane];
        } else {
#pragma unroll
            for (int j = 1; j < K; ++j) {
                const bool ge = kk >= j;
                p0 = ge ? pre[j] : p0;
                if (j + 1 < K) p1 = ge ? pre[j + 1] : p1;
            }
        }
        const float e = __builtin_fmaf(c.sp30, (float)p0, lo);
        float e1 = __builtin_fmaf(c.sp30, (float)p1, lo);
        // computed for every lane, then selected: as a conditional the compiler
        // sank the LUT read into a branch with its own LDS wait
#if NFK_E1_SEL
        asm volatile("" : "+v"(e1));
#endif
        e1 = (kk == K - 1) ? c.hi : e1;
        ek[r] = e;
        sk[r] = e1 - e;
        // wide layers (K = 16): one coordinate at a time, or the scheduler
        // interleaves the four and runs out of registers
        if constexpr (K > 8) __builtin_amdgcn_sched_barrier(0);
    }
}

// Ablation hooks for diagnostic builds (tools/ablate_build.sh; never in the
// product build): NFK_ABL_NOSTAGE drops the chunk-loop record copies,
// NFK_ABL_NOEPI replaces the spline
// epilogue by a sum.
#ifdef NFK_ABL_NOSTAGE
#define NFK_STAGE(...) ((void)0)
#else
#define NFK_STAGE(...) stage_record<kNsfWaves>(__VA_ARGS__)
#endif

// One workgroup = kNsfWaves (4) waves, one per SIMD, x 16 samples each; two
// workgroups share a CU (c3: one 51-KiB record slot + 16 KiB of x tiles), so
// one's epilogue VALU can run beside the other's MFMAs, and its barrier
// waits, prologue copies and z stores are covered by the other.
// A layer is a sequence of NP = 2 + 3 NCH phases (layer 1, layer 2, then per
// 16-coordinate chunk: searched knots, other knots, derivatives); each phase
// is a GEMM half (MFMA from the record slot) and an epilogue half (VALU on the
// accumulators).  Half-steps: GEMM of phase p = half-step 2p, its epilogue
// 2p+1, each ended by a workgroup barrier.  After the barrier ending GEMM p
// every wave's reads of the slot have returned, so phase p+1's record is
// copied into the slot; the copy overlaps epilogue p and is waited for
// (vmcnt(0)) at the barrier ending it.  The loop issues no other global
// memory operation: x is staged in the prologue and z is collected in LDS.
// Measured alternatives: two slots with one 8-wave
// workgroup per CU, lockstep or ping-pong (4-6 % slower); a persistent form
// prefetching the next tile's x into registers (no faster, SGPR spills).
__device__ __forceinline__ void stage_phase(const FusedArgs& a, const float* __restrict__ pack, int p, int offA,
                                            int offB, int offC, float4* slot, int wid, int lane) {
    if (p == 0) {
        stage_record<kNsfWaves>(pack + a.o_h1, a.blk_h1, slot, wid, lane);
    } else if (p == 1) {
        stage_record<kNsfWaves>(pack + a.o_h2, a.blk_h2, slot, wid, lane);
    } else {
        const int ch = (p - 2) / 3, part = (p - 2) - 3 * ch;
        const float* wc = pack + a.o_w3 + (int64_t)ch * a.blk_chunk * 256;
        const int off = part == 0 ? offA : (part == 1 ? offB : offC);
        NFK_STAGE(wc + off * 256, part == 2 ? a.blk_d : a.blk_w, slot, wid, lane);
    }
}

// ---- split form: records cut into sub-records of NS tiles (NfkSplit), so the
// slot shrinks to KBH NS 2 + 2 blocks and three workgroups share a CU.
template <int KBH, bool T1, int K, int HT>
struct NfkSplit {
    static constexpr int NS = KBH <= 3 ? NFK_SPLIT_NS : 2;  // tiles per sub-record
    static constexpr int NH2 = (HT + NS - 1) / NS;   // layer-2 sub-records
    static constexpr int NW = (K + NS - 1) / NS;     // W (or H) logits sub-records
    static constexpr int ND = (K - 1 + NS - 1) / NS; // derivative logits sub-records
    static constexpr int SPC = 2 * NW + ND;          // sub-records per chunk
    static constexpr int slot_blocks = KBH * NS * 2 + (T1 ? (NS + 1) / 2 : 0) + 1;
};

// Copy tiles [t0, t0 + NS) (fewer at the record's end) of the record at rec
// (nt tiles) into the slot at tile stride NS: per k-block NS x {hi, lo}
// blocks, then the tail blocks holding them, then the record's bias block.
template <int KBH, bool T1, int NS>
__device__ __forceinline__ void stage_tiles(const float* __restrict__ rec, int nt, int t0, float4* slot, int wid,
                                            int lane) {
    constexpr int NTB = T1 ? (NS + 1) / 2 : 0, NF = KBH * NS * 2, NB = NF + NTB + 1;
    const int nts = (nt - t0) < NS ? (nt - t0) : NS;
    const uint32_t base = lds_addr(slot);
    for (int i = wid; i < NB; i += kNsfWaves) {
        int src;
        if (i < NF) {
            const int kb = i / (2 * NS), r = i - kb * 2 * NS;
            if ((r >> 1) >= nts) continue;
            src = (kb * nt + t0 + (r >> 1)) * 2 + (r & 1);
        } else if (i < NF + NTB) {
            src = KBH * nt * 2 + (t0 >> 1) + (i - NF);
        } else {
            src = KBH * nt * 2 + (T1 ? (nt + 1) / 2 : 0);
        }
        dma_blk(rec + (int64_t)src * 256, lane, base + i * 1024);
    }
}

// Block b of an NS-tile sub-record (tiles [t0, t0 + NS) of a record with nt
// tiles, at tile stride NS per k-block, then its tail blocks and the record's
// bias block: stage_tiles' slot layout) -> block of the record; -1 for none.
__host__ __device__ inline int subrec_tile_src(int b, int kbh, int t1, int ns, int nt, int t0) {
    const int nf = kbh * ns * 2, ntb = t1 ? (ns + 1) / 2 : 0;
    const int nts = (nt - t0) < ns ? (nt - t0) : ns;
    if (b < nf) {
        const int kb = b / (2 * ns), r = b - kb * 2 * ns;
        if ((r >> 1) >= nts) return -1;
        return (kb * nt + t0 + (r >> 1)) * 2 + (r & 1);
    }
    if (b < nf + ntb) return kbh * nt * 2 + (t0 >> 1) + (b - nf);
    if (b == nf + ntb) return kbh * nt * 2 + (t1 ? (nt + 1) / 2 : 0);
    return -1;
}

// Stage sub-record s of the split sequence: layer 1 (whole), NH2 layer-2
// sub-records, then per chunk NW searched-knot, NW other-knot and ND
// derivative sub-records.
template <int KBH, bool T1, int K, int HT>
__device__ __forceinline__ void stage_split(const FusedArgs& a, const float* __restrict__ pack, int s, int offA,
                                            int offB, int offC, float4* slot, int wid, int lane) {
    using S = NfkSplit<KBH, T1, K, HT>;
    if (s == 0) {
        stage_record<kNsfWaves>(pack + a.o_h1, a.blk_h1, slot, wid, lane);
        return;
    }
    if (s <= S::NH2) {
        stage_tiles<KBH, T1, S::NS>(pack + a.o_h2, HT, (s - 1) * S::NS, slot, wid, lane);
        return;
    }
#ifdef NFK_ABL_NOSTAGE
    return;  // diagnostic: chunk-loop sub-records never copied
#endif
    const int u = s - 1 - S::NH2, ch = u / S::SPC, v = u - ch * S::SPC;
    const float* wc = pack + a.o_w3 + (int64_t)ch * a.blk_chunk * 256;
    if (v < S::NW)
        stage_tiles<KBH, T1, S::NS>(wc + offA * 256, K, v * S::NS, slot, wid, lane);
    else if (v < 2 * S::NW)
        stage_tiles<KBH, T1, S::NS>(wc + offB * 256, K, (v - S::NW) * S::NS, slot, wid, lane);
    else
        stage_tiles<KBH, T1, S::NS>(wc + offC * 256, K - 1, (v - 2 * S::NW) * S::NS, slot, wid, lane);
}

// GEMM over all parts J, J+1, ... of an NT-tile record: each part is followed
// by step(last) (barrier, next copy; if not last, wait for it).
template <int KBH, bool T1, int NT, int NS, int J, class Step>
__device__ __forceinline__ void gemm_parts(const h8 (&bh)[KBH], const h8 (&bl)[KBH], h4 btail,
                                           const float4* slot, int lane, f32x4 (&acc)[NT], Step&& step) {
    constexpr int T0 = J * NS;
    constexpr int N = (NT - T0) < NS ? (NT - T0) : NS;
    constexpr bool last = T0 + NS >= NT;
    gemm_h<KBH, T1, N, NS, T0, NT>(bh, bl, btail, slot, lane, acc);
    step(last);
    if constexpr (!last) gemm_parts<KBH, T1, NT, NS, J + 1>(bh, bl, btail, slot, lane, acc, step);
}

#ifndef NFK_NSF_WPE
#define NFK_NSF_WPE 2  // waves per SIMD the register budget is sized for
#endif

// CHAIN (split form only): a.nlayers layers in one launch.  The wave's x rows
// stay in its LDS tile from the first layer to the last (layer l reads and
// overwrites the tile columns a.cmaps gives it), log|det| is carried in a
// register and the status bits in LDS words, and the layer-1 record of layer l + 1 is copied
// during the last epilogue of layer l: one prologue and one tail per chain.
template <int KBH, bool T1, int K, bool INV, bool SPLIT, bool CHAIN = false>
__global__ __launch_bounds__(64 * kNsfWaves, SPLIT ? NFK_NSF_WPE_SPLIT : NFK_NSF_WPE) void k_fused_nsf(FusedArgs a) {
    static_assert(SPLIT || !CHAIN, "the chain form is a split-form kernel");
    // the arguments through a pointer the chain form re-derives opaquely at
    // every layer, so values loaded from them are not hoisted out of the layer
    // loop (kept live across it, they spilled)
    using ArgsK = const __attribute__((address_space(4))) FusedArgs;
    ArgsK* A = (ArgsK*)__builtin_amdgcn_kernarg_segment_ptr();  // a is the only argument: offset 0
    (void)a;
    constexpr int HT = 2 * KBH + (T1 ? 1 : 0);
    constexpr int DN = K - 1 > 0 ? K - 1 : 1;
    using SP = NfkSplit<KBH, T1, K, HT>;
    // pipelined chunk schedule: split form with two sub-records per W/H/D record
    constexpr bool PIPE = SPLIT && NFK_SPLIT_PIPE && SP::NW == 2 && SP::ND == 2;
    // packed knot prefixes, except in the inverse chain (it spills with them)
    constexpr bool PK2 = !(INV && CHAIN);
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4, sl = lane & 15;
    const int D = A->n_lo + A->n_up;
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    float4* slot = lds4;
    const int NL = CHAIN ? A->nlayers : 1;
    int32_t* m_up_in = reinterpret_cast<int32_t*>(lds4 + A->slot_blocks * 64);
    int32_t* m_up_out = m_up_in + A->n_up;
    int32_t* m_lo_in = m_up_out + A->n_up;
    int32_t* m_lo_out = m_lo_in + A->n_lo;
    int32_t* m_src = m_lo_out + A->n_lo;  // split form: input column of each output column
    // chain form: the maps region holds the status word of each layer (OR-ed
    // by the waves), then A->cmaps as bytes ((NL + 1) D, D <= 128): small
    // enough that three workgroups still share a CU
    int32_t* const cst = reinterpret_cast<int32_t*>(lds4 + A->slot_blocks * 64);
    uint8_t* const cm = reinterpret_cast<uint8_t*>(cst + NL);
    const uint8_t* c_lo = cm;  // this layer's lower / upper input columns
    const uint8_t* c_up = cm;
    const uint8_t* const c_src = cm + NL * (A->n_lo + A->n_up);
    // maps by index, in either form
    auto lo_map = [&](int k) { return CHAIN ? (int)c_lo[k] : m_lo_in[k]; };
    auto up_map = [&](int j) { return CHAIN ? (int)c_up[j] : m_up_in[j]; };
    auto src_map = [&](int o) { return CHAIN ? (int)c_src[o] : m_src[o]; };
    const int XL = 32 * A->KB1;  // lower-x tile row length (n_lo padded to the k-blocks)
    const int XU = A->xup;       // upper-x tile row length (n_up padded to 4)
    // split form: xlo is this wave's [16][XS] tile of whole x rows (input column
    // order, row stride XS = D + 1); the spline writes z's upper values over the
    // x values they replace
    const int XS = D + 1;
    float* xlo = reinterpret_cast<float*>(lds4 + A->slot_blocks * 64 +
                                          (CHAIN ? (4 * NL + (NL + 1) * D + 15) / 16
                                                 : (SPLIT ? 3 * D + 3 : 2 * D + 3) / 4)) +
                 wid * A->xtile;
    float* xup = xlo + 16 * XL;
    // this wave's bin lookup table: K + 1 rows of 64 lanes, after all x tiles
    int* scr = reinterpret_cast<int*>(xlo + (kNsfWaves - wid) * A->xtile) + wid * K * 64;
    const float* pk = CHAIN ? A->packs[0] : A->pack;  // this layer's pack
    int lyr = 0;                                    // chain: the layer running
    const int NP = 2 + 3 * A->NCH;
    // execution order of the three records of a chunk: searched knots, other knots, derivatives
    const int offA = INV ? A->blk_w : 0, offB = INV ? 0 : A->blk_w, offC = 2 * A->blk_w;
    const int64_t b0 = ((int64_t)blockIdx.x * kNsfWaves + wid) * 16;
    const int64_t rem = A->batch - b0;
    const int nrows = rem <= 0 ? 0 : (rem < 16 ? (int)rem : 16);
    const bool row_ok = sl < nrows;
    h8 bh[KBH], bl[KBH];  // B operands (activations) of the current product
    h4 btail = h4{0, 0, 0, 0};
    NfkTrace tr;
    (void)tr;
    NFK_MARK(tr);  // start

    // Sub-record sequence: whole records (sr = phase) or the split form's
    // sub-records.  gemm_end ends a GEMM (part): LDS reads retired, barrier,
    // the next sub-record's copy issued; inside a split record it also waits
    // for that copy.  epi_end ends an epilogue: the copy has landed, barrier.
    const int NSR = SPLIT ? 1 + SP::NH2 + A->NCH * SP::SPC : NP;
    int sr = 0;
    auto gemm_end = [&](bool last) {
        NFK_MARK(tr);  // GEMM issued
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        NFK_MARK(tr);  // barrier passed
        if (sr + 1 < NSR) {
            if constexpr (SPLIT)
                stage_split<KBH, T1, K, HT>(a, pk, sr + 1, offA, offB, offC, slot, wid, lane);
            else
                stage_phase(a, pk, sr + 1, offA, offB, offC, slot, wid, lane);
        } else if (CHAIN && lyr + 1 < NL) {
            // the next layer's layer-1 record (its pack pointer loaded here: no
            // register carries it through the layer)
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
        NFK_MARK(tr);  // epilogue issued
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        NFK_MARK(tr);  // barrier passed
    };
    // a GEMM over a whole record (acc: its NT tiles), then the step(s)
    auto gemm_rec = [&](auto& acc) {
        constexpr int N = sizeof(acc) / sizeof(f32x4);
        if constexpr (SPLIT) {
            gemm_parts<KBH, T1, N, SP::NS, 0>(bh, bl, btail, slot, lane, acc, gemm_end);
        } else {
            gemm_h<KBH, T1, N>(bh, bl, btail, slot, lane, acc);
            gemm_end(true);
        }
    };

    // ---- prologue: index maps, pack scale factors, the log|det| being
    // accumulated and the status word (plain loads, before any DMA is in
    // flight, so the end of the kernel does not wait on them), then the
    // layer-1 record and both x tiles by LDS-DMA
    if constexpr (SPLIT) {
        // split form: whole x rows first (16-B LDS-DMA, no dependency on the
        // maps; rows past the batch re-read row 0 of the tile), the layer-1
        // record, then the maps by plain loads; one wait for all of it
        if (nrows > 0) {
            // one 4-B-per-lane DMA per 64 columns of a row: rows land at the odd
            // stride XS = D + 1, so the per-sample reads below are bank-conflict free
            const uint32_t base = lds_addr(xlo);
            for (int r = 0; r < 16; ++r) {
                const float* src = A->x + (b0 + (r < nrows ? r : 0)) * A->ldx;
                for (int c0 = 0; c0 < D; c0 += 64)
                    if (c0 + lane < D) dma4(src + c0 + lane, base + (r * XS + c0) * 4);
            }
        }
        stage_phase(a, pk, 0, offA, offB, offC, slot, wid, lane);
        if constexpr (CHAIN) {
            for (int i = threadIdx.x; i < (NL + 1) * D; i += 64 * kNsfWaves) cm[i] = (uint8_t)A->cmaps[i];
            if ((int)threadIdx.x < NL) cst[threadIdx.x] = 0;
        } else {
            for (int i = threadIdx.x; i < A->n_up; i += 64 * kNsfWaves) {
                const int ui = A->up_in[i], uo = A->up_out[i];
                m_up_in[i] = ui;
                m_up_out[i] = uo;
                m_src[uo] = ui;
            }
            for (int i = threadIdx.x; i < A->n_lo; i += 64 * kNsfWaves) {
                const int li = A->lo_in[i], lo = A->lo_out[i];
                m_lo_in[i] = li;
                m_lo_out[i] = lo;
                m_src[lo] = li;
            }
        }
    } else {
        for (int i = threadIdx.x; i < A->n_up; i += 64 * kNsfWaves) {
            m_up_in[i] = A->up_in[i];
            m_up_out[i] = A->up_out[i];
        }
        for (int i = threadIdx.x; i < A->n_lo; i += 64 * kNsfWaves) {
            m_lo_in[i] = A->lo_in[i];
            m_lo_out[i] = A->lo_out[i];
        }
    }
    // status words: lane l holds layer l's (chain form: one per layer)
    // (chain form: read in the tail instead, where it costs no register
    // across the layer loop)
    int st_prev = (!CHAIN && A->status != nullptr && lane == 0) ? A->status[0] : 0;
    const float ld_prev = (q == 0 && row_ok && A->mode == 2) ? A->logdet[b0 + sl] : 0.0f;
    // split form: this lane's layer-1 columns of k-block 0 (8q + j), read from
    // the global map now so the first operand reads need no map round trip
    // (chain form: from the LDS maps, per layer)
    int lo_c0[8];
    if constexpr (SPLIT && !CHAIN) {
#pragma unroll
        for (int j = 0; j < 8; ++j) lo_c0[j] = (8 * q + j < A->n_lo) ? A->lo_in[8 * q + j] : -1;
    }
    if constexpr (!SPLIT) {
        __syncthreads();  // maps visible (no DMA in flight yet)
        stage_phase(a, pk, 0, offA, offB, offC, slot, wid, lane);
        if (nrows > 0) gather_x(A->x, A->ldx, b0, nrows, m_lo_in, A->n_lo, XL, xlo, lane);
        if (nrows > 0) gather_x(A->x, A->ldx, b0, nrows, m_up_in, A->n_up, XU, xup, lane);
    }
    dma_barrier();
    NFK_MARK(tr);  // prologue done

    // log|det| of this lane's sample (lane group 0): the stored value (mode 2)
    // plus the layer sums one by one, the order of a launch per layer
    float ld_acc = ld_prev;
    uint64_t st_bits = 0;  // status bits (chain form: per layer in the LDS words cst)
    for (int l = 0; l < NL; ++l) {
    if constexpr (CHAIN) {
        asm volatile("" : "+s"(A));
        lyr = l;
        pk = A->packs[l];
        c_lo = cm + l * D;
        c_up = c_lo + A->n_lo;
        sr = 0;
    }
    const FusedConst c = *(const FusedConst*)&A->c;  // by value (SGPRs); per layer: see A
    const float un1 = pk[3], un2 = pk[4], un3 = pk[5];
        bool any_in = false, any_nd = false;

        // layer-1 B operand of k-block kb: lower coordinates 32 kb + 8 q .. + 7 of
        // sample sl (zero past n_lo in the split form; the whole form's padding
        // columns hold a valid x, their weights are zero)
        auto x_operand = [&](int kb, float4& u, float4& v) {
            if constexpr (SPLIT) {
                float e[8];
    #pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int k = 32 * kb + 8 * q + j;
                    // map and x reads unconditional (clamped), then selected: a
                    // guarded read became a branch with its own LDS wait
                    const bool ok = k < A->n_lo;
                    const int m = lo_map(ok ? k : 0);
                    const int col = (kb == 0 && !CHAIN) ? lo_c0[j] : (ok ? m : -1);
                    const float xv0 = xlo[sl * XS + (col >= 0 ? col : 0)];
                    e[j] = col >= 0 ? xv0 : 0.0f;
                }
                u = make_float4(e[0], e[1], e[2], e[3]);
                v = make_float4(e[4], e[5], e[6], e[7]);
            } else {
                const float4* xr = reinterpret_cast<const float4*>(xlo + sl * XL + 32 * kb + 8 * q);
                u = xr[0], v = xr[1];
            }
        };
        // tile position of upper coordinate j of sample sl
        auto up_pos = [&](int j) { return SPLIT ? sl * XS + up_map(j) : sl * XU + j; };

        // ---- phase 0: layer 1, fp16 split.  x has any magnitude, so each
        // wave scales its tile by a power of two 2^sx that puts max|x| just under
        // 2^14 before the split; acc = 2^(s1+sx) W1 x.
        f32x4 h1[HT];
        float unx;
        {
            float mx = 0.0f;
            float4 u0, v0;  // k-block 0's operand, read once
            for (int kb = 0; kb < A->KB1; ++kb) {
                float4 u, v;
                x_operand(kb, u, v);
                if (kb == 0) u0 = u, v0 = v;
                mx = fmaxf(mx, fmaxf(fmaxf(fmaxf(fabsf(u.x), fabsf(u.y)), fmaxf(fabsf(u.z), fabsf(u.w))),
                                     fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)))));
            }
    #pragma unroll
            for (int off = 16; off < 64; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));  // per sample: the 4 lanes of column sl
            int ex = 0;
            if (mx > 0.0f && mx < 3.0e38f) frexpf(mx, &ex);  // mx < 2^ex
            ex = ex < -64 ? -64 : ex;  // a tiny sample: its scale 2^(14 - ex) and bias scale stay finite
            const float sx = ldexpf(1.0f, 14 - ex);
            unx = ldexpf(un1, ex - 14);
            // accumulators start at b1 2^(s1+sx) (exact power-of-two scaling), so the
            // epilogue only multiplies by 2^-(s1+sx): the bias is read in this GEMM
            // half, before the slot is recycled
            const float4* s = slot;
            const float4* bias = s + A->KB1 * HT * 2 * 64;
            const float bsc = ldexpf(1.0f, 14 - ex) / un1;
    #pragma unroll
            for (int t = 0; t < HT; ++t) {
                const float4 bv = bias[t * 4 + q];
                h1[t] = f32x4{bv.x * bsc, bv.y * bsc, bv.z * bsc, bv.w * bsc};
            }
            for (int kb = 0; kb < A->KB1; ++kb) {
                float4 u = u0, v = v0;
                if (kb > 0) x_operand(kb, u, v);
                const float xv8[8] = {u.x * sx, u.y * sx, u.z * sx, u.w * sx, v.x * sx, v.y * sx, v.z * sx, v.w * sx};
                h8 xh, xl8;
    #pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const _Float16 hh = (_Float16)xv8[j];
                    xh[j] = hh;
                    xl8[j] = (_Float16)(xv8[j] - (float)hh);
                }
    #pragma unroll
                for (int t = 0; t < HT; ++t) {
                    const h8 ahi = __builtin_bit_cast(h8, s[((kb * HT + t) * 2) * 64 + lane]);
                    const h8 alo = __builtin_bit_cast(h8, s[((kb * HT + t) * 2 + 1) * 64 + lane]);
                    h1[t] = mfma16(alo, xh, h1[t]);
                    h1[t] = mfma16(ahi, xl8, h1[t]);
                    h1[t] = mfma16(ahi, xh, h1[t]);
                }
            }
        }
        gemm_end(true);
        // epilogue 0: tanh of acc 2^-(s1+sx), split -> layer-2 operands
        act_operands<KBH, T1, HT>(h1, -2.0f * kL2E * unx, bh, bl, btail);
        epi_end();
        // ---- phase 1: layer 2, fp16 split: h2^T = tanh(W2 . h1^T + b2)
        {
            f32x4 h2[HT];
            gemm_rec(h2);
            act_operands<KBH, T1, HT>(h2, -2.0f * kL2E * un2, bh, bl, btail);
        }
        epi_end();

        const float l2e3 = kL2E * un3;
        float ldsum = 0.0f;
        // per-coordinate state of the chunk: lane group q holds coordinates
        // jbase + 4q + r, r = 0..3, of sample sl
        int jj4[4];
        int pos4[4];  // tile position of each coordinate (clamped past n_up)
        float xv[4];
        int kb[4];
        float cw_k[4], w_k[4], ch_k[4], h_k[4];
        // epilogue A (searched knots: widths forward / heights inverse) for r in [R0, R1)
        auto epi_a = [&](const f32x4(&acc)[K], int jbase, auto r0c, auto r1c) {
            constexpr int R0 = decltype(r0c)::value, R1 = decltype(r1c)::value;
    #pragma unroll
            for (int r = R0; r < R1; ++r) {
                jj4[r] = jbase + 4 * q + r;
                const bool ok = jj4[r] < A->n_up;
                pos4[r] = up_pos(ok ? jj4[r] : 0);
                const float v = (SPLIT ? xlo : xup)[pos4[r]];
                xv[r] = ok ? v : 0.0f;
            }
            knot_phase<K, true, R0, R1, PK2>(acc, xv, c, l2e3, kb, INV ? ch_k : cw_k, INV ? h_k : w_k, scr, lane);
        };
        // epilogue B: the other knots, selected at the bin
        auto epi_b = [&](const f32x4(&acc)[K], auto r0c, auto r1c) {
            constexpr int R0 = decltype(r0c)::value, R1 = decltype(r1c)::value;
            knot_phase<K, false, R0, R1, PK2>(acc, xv, c, l2e3, kb, INV ? cw_k : ch_k, INV ? w_k : h_k, scr, lane);
        };
        // epilogue C: derivatives of the bin, evaluate, log|det|
        auto epi_c = [&](const f32x4(&accd)[DN], auto r0c, auto r1c) {
            constexpr int R0 = decltype(r0c)::value, R1 = decltype(r1c)::value;
    #ifdef NFK_ABL_NOEPI
    #pragma unroll
            for (int r = R0; r < R1; ++r) {
                float v = cw_k[r] + w_k[r] + ch_k[r] + h_k[r];
    #pragma unroll
                for (int t = 0; t < DN; ++t) v += accd[t][r];
                if (jj4[r] < A->n_up) (SPLIT ? xlo : xup)[pos4[r]] = v;
                ldsum += v;
                any_in = true;
            }
            if (false)
    #endif
    #pragma unroll
            for (int r = R0; r < R1; ++r) {
                // padded derivative index j+1 holds logit j (utils.py:36-39):
                // raw_k = logit k-1, raw_k1 = logit k
                const int k = kb[r];
                float raw_k = accd[0][r], raw_k1 = accd[0][r];
                if (NFK_LUT) {
                    // row j = logit j; raw_k is unused at k = 0, raw_k1 at k = K - 1
                    float* fs = reinterpret_cast<float*>(scr);
    #pragma unroll
                    for (int j = 0; j < K - 1; ++j) fs[j * 64 + lane] = accd[j][r];
                    raw_k = fs[(k > 0 ? k - 1 : 0) * 64 + lane];
                    raw_k1 = fs[(k < K - 1 ? k : K - 2) * 64 + lane];
                } else {
    #pragma unroll
                    for (int j = 1; j < K - 1; ++j) {
                        raw_k = (k >= j + 1) ? accd[j][r] : raw_k;
                        raw_k1 = (k >= j) ? accd[j][r] : raw_k1;
                    }
                }
                // d = min_d + softplus(softplus(D)) (flows.py:235, utils.py:82), only
                // at the two knots the bin uses; the padded ends are the constant d_edge
                // both evaluated, then selected: as a conditional the compiler
                // branches around the exp/log under an exec mask
                const float dv_k = nfk_deriv_lean_s(raw_k, l2e3, c.min_d);
                const float dv_k1 = nfk_deriv_lean_s(raw_k1, l2e3, c.min_d);
                const float d_k = (k == 0) ? c.d_edge : dv_k;
                const float d_k1 = (k == K - 1) ? c.d_edge : dv_k1;
                const float x = xv[r];
                // one reciprocal of the bin width for delta and theta
                const float rw = nfk_rcp_fast(w_k[r]);
                const float delta = h_k[r] * rw;
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
                    th = (x - cw_k[r]) * rw;
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
                const bool live = jj4[r] < A->n_up && row_ok;
                out = inside ? out : x;
                if (jj4[r] < A->n_up) (SPLIT ? xlo : xup)[pos4[r]] = out;  // z collected in the tile
                ldsum += (inside && live) ? lad : 0.0f;
                any_in |= inside && live;
                any_nd |= nd && inside && live;
            }
        };
        using I0 = std::integral_constant<int, 0>;
        using I2 = std::integral_constant<int, 2>;
        using I4 = std::integral_constant<int, 4>;

        if constexpr (PIPE) {
            // Pipelined split schedule (two sub-records per record): the copy of a
            // record's second sub-record is covered by half (two coordinates) of
            // the previous phase's epilogue, the copy of the next record's first
            // sub-record by the other half.  Each phase's accumulators stay live
            // through the first GEMM part of the next phase.
            constexpr int NSP = SP::NS;
            f32x4 accd[DN];
            for (int ch = 0; ch < A->NCH; ++ch) {
                const int jbase = 16 * ch;
                f32x4 accA[K], accB[K];
                gemm_h<KBH, T1, NSP, NSP, 0, K>(bh, bl, btail, slot, lane, accA);
                gemm_end(true);
                if (ch > 0) epi_c(accd, I2{}, I4{});  // previous chunk, coordinates 2, 3
                epi_end();
                gemm_h<KBH, T1, K - NSP, NSP, NSP, K>(bh, bl, btail, slot, lane, accA);
                gemm_end(true);
                epi_a(accA, jbase, I0{}, I2{});
                epi_end();
                gemm_h<KBH, T1, NSP, NSP, 0, K>(bh, bl, btail, slot, lane, accB);
                gemm_end(true);
                epi_a(accA, jbase, I2{}, I4{});
                epi_end();
                gemm_h<KBH, T1, K - NSP, NSP, NSP, K>(bh, bl, btail, slot, lane, accB);
                gemm_end(true);
                epi_b(accB, I0{}, I2{});
                epi_end();
                gemm_h<KBH, T1, NSP, NSP, 0, DN>(bh, bl, btail, slot, lane, accd);
                gemm_end(true);
                epi_b(accB, I2{}, I4{});
                epi_end();
                gemm_h<KBH, T1, DN - NSP, NSP, NSP, DN>(bh, bl, btail, slot, lane, accd);
                gemm_end(true);
                epi_c(accd, I0{}, I2{});
                epi_end();
            }
            epi_c(accd, I2{}, I4{});  // last chunk, coordinates 2, 3
        } else {
            for (int ch = 0; ch < A->NCH; ++ch) {
                const int jbase = 16 * ch;
                {
                    f32x4 acc[K];
                    gemm_rec(acc);
                    epi_a(acc, jbase, I0{}, I4{});
                }
                epi_end();
                {
                    f32x4 acc[K];
                    gemm_rec(acc);
                    epi_b(acc, I0{}, I4{});
                }
                epi_end();
                {
                    f32x4 accd[DN];
                    gemm_rec(accd);
                    epi_c(accd, I0{}, I4{});
                }
                epi_end();
            }
        }



    // end of the layer: its log|det| added to the running sum (the order of a
    // per-layer launch sequence), its status bits kept for the tail
    {
        float v = ldsum;
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        ld_acc = ld_acc + v;  // mode 1: ld_prev = 0
        const int bits = (__any(any_in) ? NFK_ST_INSIDE_SEEN : 0) | (__any(any_nd) ? NFK_ST_NEG_DISC : 0);
        if constexpr (CHAIN) {
            if (lane == 0 && bits != 0) atomicOr(cst + l, bits);  // LDS word of layer l
        } else {
            st_bits |= (uint64_t)bits;
        }
    }
    }  // layers

    // ---- z rows of this wave (upper from the tile, lower = identity copy), log|det|
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (SPLIT) {
        // whole z rows, 16 B per lane: output column o takes tile column m_src[o]
        const int D4 = D >> 2;
        if (!CHAIN || A->z != nullptr)
        for (RowWalk w(lane, D4); w.r < nrows; w.next()) {
            const float* row = xlo + w.r * XS;
            const int o = 4 * w.k;
            *reinterpret_cast<float4*>(A->z + (b0 + w.r) * A->ldz + o) =
                make_float4(row[src_map(o)], row[src_map(o + 1)], row[src_map(o + 2)], row[src_map(o + 3)]);
        }
    } else {
        for (RowWalk w(lane, A->n_up); w.r < nrows; w.next())
            A->z[(b0 + w.r) * A->ldz + m_up_out[w.k]] = xup[w.r * XU + w.k];
        for (RowWalk w(lane, A->n_lo); w.r < nrows; w.next())
            A->z[(b0 + w.r) * A->ldz + m_lo_out[w.k]] = xlo[w.r * XL + w.k];
    }
    if (q == 0 && row_ok && A->mode != 0) A->logdet[b0 + sl] = ld_acc;
    if constexpr (CHAIN) {
        // prior epilogue (NormalizingFlowModel.evaluate, models.py:37-40, with the
        // isotropic Normal prior): log N(z; 0, s^2 I) + log|det| from the tile
        // row, the 4 lanes of sample sl summing output columns 4(q + 4i) .. + 3
        // as k_normal_lp4 does (y = z / s)
        if (A->log_prob != nullptr) {
            const float* row = xlo + sl * XS;
            const float il = A->prior_inv_scale;
            float m = 0.0f;
            for (int g = q; g < (D >> 2); g += 4) {
                const int o = 4 * g;
                const float y0 = row[src_map(o)] * il, y1 = row[src_map(o + 1)] * il;
                const float y2 = row[src_map(o + 2)] * il, y3 = row[src_map(o + 3)] * il;
                m += (y0 * y0 + y1 * y1) + (y2 * y2 + y3 * y3);
            }
            m += __shfl_xor(m, 16, 64);
            m += __shfl_xor(m, 32, 64);
            const float lp = -0.5f * (A->prior_c2pi + m) - A->prior_hld;
            if (q == 0 && row_ok) A->log_prob[b0 + sl] = lp + ld_acc;
            // a NaN in z (m NaN): the prior's argument validation raises (NFK_ST_NAN_Z)
            if (__any(row_ok && m != m) && lane == 0) atomicOr(cst, NFK_ST_NAN_Z);
        }
    }
    if constexpr (CHAIN) {
        // the workgroup's status bits of every layer (LDS words), one global
        // atomic per layer and workgroup where they add a bit
        __syncthreads();
        if (A->status != nullptr && (int)threadIdx.x < NL) {
            const int bits = cst[threadIdx.x];
            if (bits != 0 && (A->status[threadIdx.x] & bits) != bits) atomicOr(A->status + threadIdx.x, bits);
        }
    } else if (A->status != nullptr) {
        const int bits = (int)st_bits;
        if (lane == 0 && bits != 0 && (st_prev & bits) != bits) atomicOr(A->status, bits);
    }
#ifdef NFK_TRACE
    NFK_MARK(tr);  // end
    nfk_trace_flush(tr, A->trace, wid, lane);
#endif
}

template <int KBH, int T1, int K>
int launch_fused(const FusedArgs& a, size_t lds, bool inv, bool split, bool chain, hipStream_t st) {
    const int64_t per_block = (int64_t)kNsfWaves * 16;
    const int64_t blocks = (a.batch + per_block - 1) / per_block;
    if (blocks == 0) return 0;
    const dim3 g((unsigned)blocks), b(64 * kNsfWaves);
    if (chain) {
        if (inv)
            hipLaunchKernelGGL((k_fused_nsf<KBH, T1 != 0, K, true, true, true>), g, b, lds, st, a);
        else
            hipLaunchKernelGGL((k_fused_nsf<KBH, T1 != 0, K, false, true, true>), g, b, lds, st, a);
    } else if (split) {
        if (inv)
            hipLaunchKernelGGL((k_fused_nsf<KBH, T1 != 0, K, true, true>), g, b, lds, st, a);
        else
            hipLaunchKernelGGL((k_fused_nsf<KBH, T1 != 0, K, false, true>), g, b, lds, st, a);
    } else {
        if (inv)
            hipLaunchKernelGGL((k_fused_nsf<KBH, T1 != 0, K, true, false>), g, b, lds, st, a);
        else
            hipLaunchKernelGGL((k_fused_nsf<KBH, T1 != 0, K, false, false>), g, b, lds, st, a);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

// explicit instantiation: definitions live in nfk_fused_kb<KBH>.hip (one TU
// per hidden k-block count so make -j compiles them in parallel); nfk_fused.hip
// sees only the extern declarations.
#define NFK_FUSED_INSTANCE(KBH, T1, K) \
    template int launch_fused<KBH, T1, K>(const FusedArgs& a, size_t lds, bool inv, bool split, bool chain, \
                                          hipStream_t st);
#define NFK_FUSED_EXTERN(KBH, T1, K) \
    extern template int launch_fused<KBH, T1, K>(const FusedArgs& a, size_t lds, bool inv, bool split, \
                                                 bool chain, hipStream_t st);

// ---- recompute + VJP form (nfk_fused_vjp.hip): the layer's records in the
// 8-coordinate (wide = 1) layout re-cut into sub-records of kVNS output tiles
// (layer 1 whole), each padded to SB blocks, double-buffered in two LDS slots.
// Stream order: layer 1, NP2 layer-2 parts, then per 8-coordinate chunk the
// W (NPW parts), H (NPW) and D (NPD) records.
constexpr int kVNS = 2;
struct VjpDims {
    int HT, NP2, KW, KD, NPW, NPD, SPC, B1, BP, SB;
};
__host__ __device__ constexpr VjpDims vjp_dims(int KBH, int T1, int K) {
    VjpDims d{};
    d.HT = 2 * KBH + (T1 ? 1 : 0);
    d.NP2 = (d.HT + kVNS - 1) / kVNS;
    d.KW = (K + 1) / 2;
    d.KD = K / 2;
    d.NPW = (d.KW + kVNS - 1) / kVNS;
    d.NPD = (d.KD + kVNS - 1) / kVNS;
    d.SPC = 2 * d.NPW + d.NPD;
    d.B1 = d.HT * 2 + 1;  // the layer-1 record with one input k-block (n_lo <= 32)
    d.BP = KBH * kVNS * 2 + (T1 ? (kVNS + 1) / 2 : 0) + 1;
    d.SB = (((d.B1 > d.BP ? d.B1 : d.BP) + 3) / 4) * 4;
    return d;
}
__host__ __device__ inline int vjp_nsub(const VjpDims& d, int nch) { return 1 + d.NP2 + nch * d.SPC; }
inline size_t vjp_lds_bytes(const VjpDims& d, int D) {
    return (size_t)2 * d.SB * 1024 + (size_t)((2 * D + 3) / 4) * 16 + (size_t)kNsfWaves * 16 * (D + 1) * sizeof(float);
}
// instantiated (KBH, T1, K) of the VJP kernel
#define NFK_VJP_SHAPES(X) X(1, 1, 4) X(1, 1, 8) X(2, 0, 4) X(2, 0, 8) X(3, 0, 4) X(3, 0, 8) X(3, 1, 4) X(3, 1, 8)
inline bool vjp_ok(int n_lo, int n_up, int H, int K) {
    if (n_lo < 1 || n_lo > 32 || n_up < 1 || n_lo + n_up > 128 || (n_lo + n_up) % 4 != 0) return false;
    const Layout L = make_layout(n_lo, n_up, H, K, 1);
    bool inst = false;
#define NFK_VJP_CHK(h, t, k) inst |= (L.KBH == h && L.T1 == t && K == k);
    NFK_VJP_SHAPES(NFK_VJP_CHK)
#undef NFK_VJP_CHK
    // two workgroups per CU at least (LDS counted in the allocation granule)
    return inst && 2 * lds_alloc(vjp_lds_bytes(vjp_dims(L.KBH, L.T1, K), n_lo + n_up)) <= (size_t)kLdsBytes;
}

// the two-tile chain (nfk_fused_chain2.hip): c3-class shapes
int launch_chain2(const FusedArgs& a, const Layout& L, int K, bool inv, hipStream_t st);
bool chain2_ok(const Layout& L, int K, int nl, bool saved = false);

// hidden widths: KBH = full fp16 k-blocks of 32, T1 = an f16 tail step of <= 4
// features (H = 32 KBH + 1..4); H <= 132
#define NFK_FUSED_KB(X) X(1, 0) X(1, 1) X(2, 0) X(2, 1) X(3, 0) X(3, 1) X(4, 0) X(4, 1)
#define NFK_FUSED_K(X, KBH, T1) X(KBH, T1, 4) X(KBH, T1, 5) X(KBH, T1, 6) X(KBH, T1, 8) X(KBH, T1, 10)

}  // namespace nfk_fused
