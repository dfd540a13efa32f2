// nfk_fused_ar.hip -- one launch per NSF_AR layer (nf/flows.py:152-209).
//
// NSF_AR splines coordinate i with the parameters of its own conditioner
// layers[i-1] (FCNN(2i, 3K-1, H), flows.py:20-35) applied to the trig features
// [cos(pi v_j / B), sin(pi v_j / B)], j < i (flows.py:172-173), of the
// layer's INPUT v = x in forward (flows.py:176-189) and of the already
// inverted OUTPUT v = x in inverse (flows.py:191-209); coordinate 0 uses
// init_param.  The reference runs dim host iterations of torch ops per layer;
// the unfused path here ran ~8 launches per coordinate.
//
// Work decomposition: a workgroup = NW waves x 16 samples.  The rows
// stay with the workgroup for the whole layer and the conditioners of the dim
// coordinates stream through it in order, so the inverse's sequential column
// loop and the forward share one structure:
//   * each conditioner is three fp16-split MFMA GEMMs (nfk_fused_impl.h
//     gemm_h: A = packed weights from LDS, B = activations in registers,
//     h^T = W act^T, the hidden features permuted so one layer's accumulators
//     are the next layer's B operands) with tanh between them;
//   * the layer-1 B operands are the trig features, kept in registers as fp16
//     hi/lo fragments in a canonical interleaved order (feature 2j = cos of
//     column j, 2j + 1 = sin), computed once per row in the forward and
//     appended column by column in the inverse; conditioner i reads the first
//     ceil(2i / 32) k-blocks of them (its weight columns are permuted to that
//     order in the pack, the k-block past 2i masked);
//   * the 3K-1 output logits of conditioner i land in a per-wave LDS slab
//     [column][sample][param]; the spline (nfk_spline.h nfk_rqs_element_lean,
//     the unfused path's element math) runs with one lane per (sample,
//     column): in forward G = 4 coordinates at once (lane group q takes
//     column i0 + q), in inverse one coordinate (every lane group computes
//     it; the result feeds the next conditioners' trig features);
//   * weights stream as uniform sub-records (SB 1-KiB blocks: NS = 3 output
//     tiles x all k-blocks x {hi, lo}, the tail step's blocks, the record's
//     bias block) through two LDS slots: the copy of sub-record s + 2 is issued
//     right after the barrier that ends the GEMM of s (one barrier per
//     sub-record), so it overlaps the GEMM of s + 1 and every epilogue between.
// log|det| is summed per sample in column order (flows.py:188, 208) and
// added to the layer's log|det| buffer like every layer kernel (modes 0/1/2).
// Status words: one per coordinate (no element inside -> RuntimeError of
// utils.py:63; negative discriminant -> AssertionError of utils.py:121).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>

#include "../../include/nfk.h"
#include "nfk_spline.h"

int nfk_set_error(const char* msg);
NfkSplineConst nfk_make_const(int K, double left, double right, double bottom, double top,
                              int tails, double min_w, double min_h, double min_d);

#include "nfk_fused_impl.h"

using namespace nfk_fused;

namespace {

#ifndef NFK_AR_NS
#define NFK_AR_NS 3
#endif
constexpr int kArNS = NFK_AR_NS;  // output tiles per sub-record (hidden widths up to 4 k-blocks)
// wider conditioners (the applications' H = 354: 11 k-blocks) take 2-tile
// sub-records, so two 46-KiB slots and the spline slabs fit one CU's LDS
#ifndef NFK_AR_NS_WIDE
#define NFK_AR_NS_WIDE 2  // (diagnostic A/B: 1-tile sub-records for the wide conditioners)
#endif
#ifdef NFK_AR_DIAG_NS2  // diagnostic: 2-tile sub-records for every width
__host__ __device__ constexpr int ar_ns_for(int) { return 2; }
#else
__host__ __device__ constexpr int ar_ns_for(int kbh) { return kbh <= 4 ? kArNS : NFK_AR_NS_WIDE; }
#endif
// waves per SIMD the register allocation targets: two for the NSF_CL-sized
// conditioners, one (512 registers: MFMA accumulators in AGPRs) for the wide
// ones, which run 4-wave workgroups only (NFK_AR_WAVES is not applied)
#ifdef NFK_AR_DIAG_ONEWAVE  // diagnostic: every width compiled for one wave per SIMD (512 registers)
__host__ __device__ constexpr int ar_min_waves(int) { return 1; }
#else
__host__ __device__ constexpr int ar_min_waves(int kbh) { return kbh <= 4 ? 2 : 1; }
#endif
// waves per workgroup, 16 samples each: 4 (one per SIMD; two independent
// workgroups share a CU, so the two waves on a SIMD run unsynchronised phases)
// or 8 (one workgroup per CU; half the weight stream per sample, but its two
// waves per SIMD run every phase in lockstep); NFK_AR_WAVES selects
constexpr int kArWavesMax = 8;
constexpr int kArMaxDim = 256;  // (the instances' layer-1 capacity KBX bounds it further)

// T1 = the hidden width's tail kind: 0 none (H = 32 KBH), 1 = 1..4 features
// (the NSF_CL kernels' f16 tail step), 2 = 5..16 features (a 16-row half tile:
// two 16x16x32 MFMAs per output tile instead of a padded 32-feature k-block)
struct ArDims {
    int KBH, T1, HT, P, NO, NS, NH, N3, SPC, NTG, KB1M, SB, PS;
};

__host__ __device__ inline ArDims ar_dims(int hidden, int K, int dim) {
    ArDims d{};
    const int kbf = hidden / 32, rem = hidden - 32 * kbf;
    d.T1 = (rem == 0 || kbf < 1) ? 0 : (rem <= 4 ? 1 : (rem <= 16 ? 2 : 0));
    d.KBH = (rem == 0 || d.T1 != 0) ? kbf : kbf + 1;
    d.HT = 2 * d.KBH + (d.T1 ? 1 : 0);
    d.P = 3 * K - 1;
    d.NO = (d.P + 15) / 16;
    d.NS = ar_ns_for(d.KBH);
    d.NH = (d.HT + d.NS - 1) / d.NS;
    d.N3 = (d.NO + d.NS - 1) / d.NS;
    d.SPC = 2 * d.NH + d.N3;
    d.NTG = d.T1 == 1 ? (d.NS + 1) / 2 : (d.T1 == 2 ? 2 * d.NS : 0);
    d.KB1M = dim > 1 ? (2 * (dim - 1) + 31) / 32 : 1;
    const int s1 = d.KB1M * d.NS * 2 + 1, s2 = d.KBH * d.NS * 2 + d.NTG + 1;
    d.SB = s1 > s2 ? s1 : s2;
    d.PS = 16 * d.NO + 4;  // slab row stride: = 4 mod 8 floats, conflict-free 16-B reads
    return d;
}
__host__ __device__ inline int64_t ar_nsub(const ArDims& d, int dim) { return (int64_t)(dim - 1) * d.SPC; }
__host__ __device__ inline int64_t ar_pack_floats(const ArDims& d, int dim) { return 256 + ar_nsub(d, dim) * d.SB * 256; }

// columns splined per spline pass: in forward 4 (one per lane group; 2 when
// the slab row is long, K > 16), in inverse 1
__host__ __device__ constexpr int ar_group(bool inv, int ps) { return inv ? 1 : (ps <= 52 ? 4 : 2); }
inline size_t ar_lds_bytes(const ArDims& d, int dim, bool inv, int nw = kArWavesMax) {
    return (size_t)2 * d.SB * 1024 + (size_t)nw * ar_group(inv, d.PS) * 16 * d.PS * sizeof(float) +
           (size_t)(dim + 3) / 4 * 16;
}

// instantiated shapes (KBH, T1, K, KBX): KBX = layer-1 k-block capacity (dim <= 16 KBX + 1)
#define NFK_AR_SHAPES(X)                                                                        \
    X(1, 0, 4, 2)   /* golden nsfar_d4_k4 (H = 16) */                                            \
    X(1, 0, 8, 2)   /* small test shapes (H <= 32) */                                           \
    X(2, 2, 10, 4)  /* applications/input/Gaussian.yaml: dim 40, K 10, H 80 (64 + a 16 tail) */ \
    X(3, 1, 8, 4)   /* H = 100 (config.py:40), K 8, dim <= 64 */                                 \
    X(3, 1, 10, 4)  /* H = 100, K 10 */                                                           \
    X(3, 1, 32, 4)  /* config.py defaults: H = 100, K 32 (nsplines), dim <= 64 */                \
    X(11, 1, 32, 6) /* Einstein / LJ.yaml: H = 354 (11 k-blocks + 2), K 32, 32 x 3 = 96 coords */ \
    X(11, 1, 32, 11) /* Fe_*.yaml: H = 354, K 32, 54 particles x 3 = 162 coordinates (<= 177) */ \
    X(3, 1, 32, 6)  /* config.py defaults (H = 100, K 32) at 32 particles x 3 dims: dim <= 97 */ \
    NFK_AR_DIAG_SHAPES(X)
#ifndef NFK_AR_DIAG_SHAPES
#define NFK_AR_DIAG_SHAPES(X)
#endif

inline bool ar_instance(const ArDims& d, int K, int* kbx) {
#define NFK_AR_CHK(h, t, k, x)                                          \
    if (d.KBH == h && d.T1 == t && K == k && d.KB1M <= x) {             \
        *kbx = x;                                                        \
        return true;                                                     \
    }
    NFK_AR_SHAPES(NFK_AR_CHK)
#undef NFK_AR_CHK
    return false;
}

// waves per workgroup of an instance (the wide conditioners: 4)
inline int ar_waves(const ArDims& d) {
    static const int nw_env = [] {
        const char* e = std::getenv("NFK_AR_WAVES");
        return (e != nullptr && e[0] == '8') ? 8 : 4;
    }();
    return ar_min_waves(d.KBH) == 1 ? 4 : nw_env;
}

inline bool ar_ok(int dim, int hidden, int K) {
    if (dim < 2 || dim > kArMaxDim || hidden < 1 || K < 2) return false;
    const ArDims d = ar_dims(hidden, K, dim);
    int kbx;
    if (!ar_instance(d, K, &kbx)) return false;
    // both directions fit one workgroup per CU at the waves a launch uses
    const int nw = ar_waves(d);
    return ar_lds_bytes(d, dim, false, nw) <= (size_t)kLdsBytes && ar_lds_bytes(d, dim, true, nw) <= (size_t)kLdsBytes;
}

// ---------------------------------------------------------------------------
// pack: header block (maxima, unscale factors, init_param), then the
// sub-record stream of conditioners 1 .. dim-1 (layer 1, layer 2, output
// layer), each sub-record padded to SB blocks.
struct ArPackArgs {
    const float* const* w;  // (dim-1) x {W1, b1, W2, b2, W3, b3}
    const float* init;      // init_param [3K-1]
    float* out;
    int dim, H, K;
    ArDims d;
};

__global__ __launch_bounds__(256) void k_ar_max(ArPackArgs a) {
    const int i = 1 + (int)blockIdx.y;  // conditioner
    const float* const* w = a.w + (int64_t)(i - 1) * 6;
    const int64_t n1 = (int64_t)a.H * 2 * i, n2 = (int64_t)a.H * a.H, n3 = (int64_t)a.d.P * a.H;
    float m1 = 0.0f, m2 = 0.0f, m3 = 0.0f;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n1 + n2 + n3;
         g += (int64_t)gridDim.x * blockDim.x) {
        if (g < n1)
            m1 = fmaxf(m1, fabsf(w[0][g]));
        else if (g < n1 + n2)
            m2 = fmaxf(m2, fabsf(w[2][g - n1]));
        else
            m3 = fmaxf(m3, fabsf(w[4][g - n1 - n2]));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        m1 = fmaxf(m1, __shfl_xor(m1, off, 64));
        m2 = fmaxf(m2, __shfl_xor(m2, off, 64));
        m3 = fmaxf(m3, __shfl_xor(m3, off, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        unsigned int* h = reinterpret_cast<unsigned int*>(a.out);
        atomicMax(h, __float_as_uint(m1));
        atomicMax(h + 1, __float_as_uint(m2));
        atomicMax(h + 2, __float_as_uint(m3));
    }
}

__device__ int ar_scale_exp(float maxw) {  // 2^s max|W| in [2^14, 2^15)
    if (!(maxw > 0.0f) || !(maxw < 3.0e38f)) return 0;
    int e;
    frexpf(maxw, &e);
    return 15 - e;
}

// Word wl of block blk of a sub-record holding tiles [T0, T0 + NS) of an
// nt-tile record over a kbn-k-block contraction (val(t, row, k): the
// unscaled weight of row `row` of tile t at contraction index k, 0 outside),
// then (t1) its tail block over contraction indices 32 kbn + 0..3 and the
// record's bias block [tile][row].  Block order and word layout are those
// gemm_h reads (nfk_fused_impl.h: k-block fragments, tail_word, bias).
template <class ValF, class BiasF>
__device__ uint32_t ar_sub_word(int ns, int blk, int wl, int kbn, int t1, int nt, int T0, float sc, float bsc,
                                ValF val, BiasF bias) {
    const int nf = kbn * ns * 2, ntg = t1 == 1 ? (ns + 1) / 2 : 0;
    if (t1 == 2 && blk >= nf) {
        // 16-feature tail: the bias block first, then per tile {A1, A2}: lane l
        // (row l & 15, lane group g = l >> 4) element j of A1 = lo (j < 4) / hi
        // (j >= 4) weight of feature 32 kbn + 4 g + (j & 3), of A2 = hi (j < 4) / 0;
        // against B1 = {hi, lo} and B2 = {hi, 0} of the half tile's 4 rows
        if (blk == nf) {  // the sub-record's own tiles (gemm_h BREL)
            const int tt = wl >> 4, t = T0 + tt, r = wl & 15;
            return __float_as_uint(tt < ns && t < nt ? bias(t, r) * bsc : 0.0f);
        }
        const int tt = blk - nf - 1;
        if (tt >= 2 * ns) return 0u;
        const int t = T0 + (tt >> 1), which = tt & 1;
        if (t >= nt) return 0u;
        const int lane = wl >> 2, g = lane >> 4, row = lane & 15, jp = 2 * (wl & 3);
        _Float16 hv[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int j = jp + e;
            const float w = val(t, row, 32 * kbn + 4 * g + (j & 3)) * sc;
            const _Float16 wh = (_Float16)w;
            if (which == 0)
                hv[e] = j < 4 ? (_Float16)(w - (float)wh) : wh;
            else
                hv[e] = j < 4 ? wh : (_Float16)0.0f;
        }
        return (uint32_t)__builtin_bit_cast(uint16_t, hv[0]) | ((uint32_t)__builtin_bit_cast(uint16_t, hv[1]) << 16);
    }
    if (blk < nf) {
        const int part = blk & 1, idx = blk >> 1, kb = idx / ns, t = T0 + (idx - kb * ns);
        if (t >= nt) return 0u;
        const int lane = wl >> 2, j = 2 * (wl & 3), k0 = 32 * kb + 8 * (lane >> 4) + j;
        return nfk_f16_part_pair(val(t, lane & 15, k0) * sc, val(t, lane & 15, k0 + 1) * sc, part);
    }
    if (blk < nf + ntg) {  // tail: (hi, hi, lo, 0) of the sub-record's tile pair (tail_word's layout)
        const int t = T0 + 2 * (blk - nf) + ((wl & 3) >> 1), lane = wl >> 2, j = 2 * (wl & 1), qq = lane >> 4;
        if (t >= nt || qq == 3) return 0u;
        const int kb0 = 32 * kbn;
        return nfk_f16_part_pair(val(t, lane & 15, kb0 + j) * sc, val(t, lane & 15, kb0 + j + 1) * sc,
                                 qq == 2 ? 1 : 0);
    }
    if (blk == nf + ntg) {  // the sub-record's own tiles (gemm_h BREL): records of > 16 tiles
        const int tt = wl >> 4, t = T0 + tt, r = wl & 15;
        return __float_as_uint(tt < ns && t < nt ? bias(t, r) * bsc : 0.0f);
    }
    return 0u;  // padding to SB blocks
}

__global__ __launch_bounds__(256) void k_ar_pack(ArPackArgs a) {
    const ArDims& d = a.d;
    uint32_t* out = reinterpret_cast<uint32_t*>(a.out);
    const unsigned int* hdr = reinterpret_cast<const unsigned int*>(a.out);
    const int s1 = ar_scale_exp(__uint_as_float(hdr[0])), s2 = ar_scale_exp(__uint_as_float(hdr[1])),
              s3 = ar_scale_exp(__uint_as_float(hdr[2]));
    const int64_t total = ar_pack_floats(d, a.dim);
    const int H = a.H, kbh = d.KBH;
    // hidden feature of row r of hidden tile t (the 16-feature half tile: 32 KBH + r)
    auto hid = [&](int t, int r) { return (d.T1 == 2 && t == 2 * kbh) ? 32 * kbh + r : hid_feature(t, r, kbh); };
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        if (g < 256) {
            if (g == 3) out[g] = __float_as_uint(ldexpf(1.0f, -(s1 + 14)));
            else if (g == 4) out[g] = __float_as_uint(ldexpf(1.0f, -(s2 + 14)));
            else if (g == 5) out[g] = __float_as_uint(ldexpf(1.0f, -(s3 + 14)));
            else if (g >= 8 && g < 8 + d.P) out[g] = __float_as_uint(a.init[g - 8]);
            else if (g >= 6) out[g] = 0u;
            continue;
        }
        const int64_t w = g - 256;
        const int64_t s = w / ((int64_t)d.SB * 256);
        const int blk = (int)((w >> 8) - s * d.SB), wl = (int)(w & 255);
        const int i = 1 + (int)(s / d.SPC), u = (int)(s - (int64_t)(i - 1) * d.SPC);
        const float* const* pw = a.w + (int64_t)(i - 1) * 6;
        uint32_t v;
        if (u < d.NH) {  // layer 1: Linear(2i, H) on the canonical trig order (k = 2j + {cos, sin})
            const float* W1 = pw[0];
            const float* b1 = pw[1];
            const int kb1 = (2 * i + 31) / 32;
            v = ar_sub_word(
                d.NS, blk, wl, kb1, 0, d.HT, d.NS * u, ldexpf(1.0f, s1), ldexpf(1.0f, s1 + 14),
                [&](int t, int r, int k) -> float {
                    const int f = hid(t, r);
                    if (f >= H || k >= 2 * i) return 0.0f;
                    return W1[(int64_t)f * 2 * i + (k & 1) * i + (k >> 1)];  // cat(cos, sin) columns
                },
                [&](int t, int r) -> float {
                    const int f = hid(t, r);
                    return f < H ? b1[f] : 0.0f;
                });
        } else if (u < 2 * d.NH) {  // layer 2: Linear(H, H)
            const float* W2 = pw[2];
            const float* b2 = pw[3];
            v = ar_sub_word(
                d.NS, blk, wl, kbh, d.T1, d.HT, d.NS * (u - d.NH), ldexpf(1.0f, s2), ldexpf(1.0f, s2 + 14),
                [&](int t, int r, int k) -> float {
                    const int f = hid(t, r);
                    return (f < H && k < H) ? W2[(int64_t)f * H + k] : 0.0f;
                },
                [&](int t, int r) -> float {
                    const int f = hid(t, r);
                    return f < H ? b2[f] : 0.0f;
                });
        } else {  // output layer: Linear(H, 3K-1), row 16 t + r = parameter (W, H, D logits in order)
            const float* W3 = pw[4];
            const float* b3 = pw[5];
            const int P = d.P;
            v = ar_sub_word(
                d.NS, blk, wl, kbh, d.T1, d.NO, d.NS * (u - 2 * d.NH), ldexpf(1.0f, s3), ldexpf(1.0f, s3 + 14),
                [&](int t, int r, int k) -> float {
                    const int p = 16 * t + r;
                    return (p < P && k < H) ? W3[(int64_t)p * H + k] : 0.0f;
                },
                [&](int t, int r) -> float {
                    const int p = 16 * t + r;
                    return p < P ? b3[p] : 0.0f;
                });
        }
        out[g] = v;
    }
}

// ---------------------------------------------------------------------------
struct ArArgs {
    const float* x;  // layer input (forward: x; inverse: z)
    const float* pack;
    float* out;      // layer output
    float* logdet;
    int32_t* status;  // [dim] words or null
    int64_t ldx, ldo, batch;
    int32_t dim, mode, sb, kb1m;
    int64_t nsr;       // sub-records in the stream
    int32_t csplit;    // forward: column ranges (1: the whole layer per workgroup)
    int64_t rblocks;   // row blocks of the batch
    float* ld_cols;    // csplit > 1: per-column log|det| terms [dim][batch], summed by k_ar_ld_sum
    float pi, bnd;     // trig features: (pi v) / B (nfk_trig_features' operation order)
    NfkSplineConst c;
};

// GEMM over the sub-records J, J + 1, ... of an NT-tile record; end() after
// each ends the sub-record (barrier, next copy) and moves to the next slot.
// busy (wave-uniform) false: a wave whose 16 rows all lie past the batch
// (small batches: 40 rows leave the fourth wave of a workgroup empty) only
// keeps the barriers and copies, not the MFMAs and their LDS reads
template <int NS, int KB, bool T1, int NT, int J, class SlotF, class EndF>
__device__ __forceinline__ void ar_parts(const h8 (&bh)[KB], const h8 (&bl)[KB], h4 bt, int lane,
                                         f32x4 (&acc)[NT], SlotF slot, EndF end, float bsc = 1.0f,
                                         bool busy = true) {
    constexpr int T0 = J * NS;
    constexpr int N = (NT - T0) < NS ? (NT - T0) : NS;
    if (busy) gemm_h<KB, T1, N, NS, T0, NT, true, T0 + NS >= NT>(bh, bl, bt, slot(), lane, acc, bsc);
    end();
    if constexpr (T0 + NS < NT) ar_parts<NS, KB, T1, NT, J + 1>(bh, bl, bt, lane, acc, slot, end, bsc, busy);
}

// The same over a hidden width with a 16-feature tail (tail kind 2): the full
// k-blocks by gemm_h (its bias block sits right after them), then per output
// tile the tail's two MFMAs on B1 = {hi, lo}, B2 = {hi, 0} of the half tile
template <int NS, int KB, int NT, int J, class SlotF, class EndF>
__device__ __forceinline__ void ar_parts16(const h8 (&bh)[KB], const h8 (&bl)[KB], h8 b1, h8 b2, int lane,
                                           f32x4 (&acc)[NT], SlotF slot, EndF end, bool busy = true) {
    constexpr int T0 = J * NS;
    constexpr int N = (NT - T0) < NS ? (NT - T0) : NS;
    if (busy) {
        const float4* sl = slot();
        gemm_h<KB, false, N, NS, T0, NT, true>(bh, bl, h4{0, 0, 0, 0}, sl, lane, acc);
        const float4* t16 = sl + (KB * NS * 2 + 1) * 64;
#pragma unroll
        for (int t = 0; t < N; ++t) {
            const h8 a1 = __builtin_bit_cast(h8, t16[(2 * t) * 64 + lane]);
            const h8 a2 = __builtin_bit_cast(h8, t16[(2 * t + 1) * 64 + lane]);
            acc[T0 + t] = mfma16(a1, b1, acc[T0 + t]);
            acc[T0 + t] = mfma16(a2, b2, acc[T0 + t]);
        }
        if constexpr (T0 + NS >= NT) mfma_result_wait();
    }
    end();
    if constexpr (T0 + NS < NT) ar_parts16<NS, KB, NT, J + 1>(bh, bl, b1, b2, lane, acc, slot, end, busy);
}

// activations of a hidden layer with a 16-feature tail: the full tiles by
// act_operands, the half tile's 4 rows per lane into B1 = {hi, lo}, B2 = {hi, 0}
template <int KBH, int HT>
__device__ __forceinline__ void act_operands16(f32x4 (&h)[HT], float c2, h8 (&bh)[KBH], h8 (&bl)[KBH], h8& b1,
                                               h8& b2) {
    h4 unused;
    act_operands<KBH, false, HT>(h, c2, bh, bl, unused);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float v = tanh_scaled(h[HT - 1][r], c2);
        const _Float16 hi = (_Float16)v;
        b1[r] = hi;
        b1[4 + r] = (_Float16)(v - (float)hi);
        b2[r] = hi;
        b2[4 + r] = (_Float16)0.0f;
    }
}

// fp16 hi/lo of two trig features (x 2^14, the activations' split scale)
__device__ __forceinline__ void trig_split(float v, float pi, float bnd, _Float16& ch, _Float16& cl, _Float16& sh,
                                           _Float16& sl) {
    const float arg = (pi * v) / bnd;
    const float c = cosf(arg) * kActScale, s = sinf(arg) * kActScale;
    ch = (_Float16)c;
    cl = (_Float16)(c - (float)ch);
    sh = (_Float16)s;
    sl = (_Float16)(s - (float)sh);
}

#ifdef NFK_AR_DIAG_DUMP  // diagnostic: conditioner 1's activations and logits of workgroup 0
__device__ float g_ar_dbg[3 * 64 * 512];
template <int HT>
__device__ void ar_dump_act(int stage, const f32x4 (&h)[HT], int kbh, int row, int q) {
    for (int t = 0; t < HT; ++t)
        for (int r = 0; r < 4; ++r) {
            const int f = hid_feature(t, 4 * q + r, kbh);
            if (f < 512) g_ar_dbg[(stage * 64 + row) * 512 + f] = h[t][r] * (1.0f / kActScale);
        }
}
extern "C" int nfk_ar_dbg_copy(float* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ar_dbg), sizeof(g_ar_dbg), 0, hipMemcpyDeviceToHost);
}
#endif

template <int KBH, int TK, int K, int KBX, bool INV, int NW>
__device__ __forceinline__ void ar_layer(ArArgs a) {
    constexpr int kArWaves = NW;
    constexpr bool T1 = TK == 1;  // the f16 4-feature tail step; TK == 2: the 16-feature tail
    constexpr int HT = 2 * KBH + (TK ? 1 : 0), P = 3 * K - 1, NO = (P + 15) / 16;
    constexpr int NS = ar_ns_for(KBH);
    constexpr int NH = (HT + NS - 1) / NS, N3 = (NO + NS - 1) / NS, SPC = 2 * NH + N3;
    constexpr int NTG = TK == 1 ? (NS + 1) / 2 : (TK == 2 ? 2 * NS : 0);
    constexpr int PS = 16 * NO + 4, G = ar_group(INV, PS);
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4, sl = lane & 15;
    const int D = a.dim;
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    float4* const slot0 = lds4;
    float4* const slot1 = lds4 + a.sb * 64;
    float* const scr = reinterpret_cast<float*>(lds4 + 2 * a.sb * 64) + wid * (G * 16 * PS);
    int* const cst = reinterpret_cast<int*>(reinterpret_cast<float*>(lds4 + 2 * a.sb * 64) + kArWaves * G * 16 * PS);
    // column range of this workgroup: the forward's conditioners are
    // independent given x, so a small batch splits them over workgroups.
    // Split grids are XCD-affine: blocks b and b + 8 share an XCD (round-robin
    // dispatch, MI355X_MICROARCH.md), so virtual id v = (b % 8) G/8 + b / 8
    // puts the row blocks of one column range on one XCD, whose L2 then
    // fetches that range's weights once (G padded to a multiple of 8)
    int sp = 0;
    int64_t rbk = blockIdx.x;
    if (a.csplit > 1) {
        const int64_t v = (int64_t)(blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
        if (v >= a.rblocks * a.csplit) return;  // padding workgroup (uniform: before any barrier)
        sp = (int)(v / a.rblocks);
        rbk = v - (int64_t)sp * a.rblocks;
    }
    const int i_lo = (int)(((int64_t)sp * D) / a.csplit), i_hi = (int)(((int64_t)(sp + 1) * D) / a.csplit);
    const int64_t b0 = (rbk * kArWaves + wid) * 16;
    const bool row_ok = b0 + sl < a.batch;
    const int64_t brow = row_ok ? b0 + sl : a.batch - 1;  // rows past the batch re-read the last one
    // every wave runs the GEMMs, rows or not: skipping them in a row-less wave
    // (a branch around each gemm_h) cost the register instances 28-1,600 VGPR
    // spills (k_fused_ar_s and k_fused_cl skip them)
    constexpr bool busy = true;

    // the next sub-record st_s (conditioner st_i, part st_u) into slot st_s & 1;
    // layer-1 sub-records hold ceil(2i / 32) k-blocks.  Called once per
    // sub-record in stream order, so a cursor replaces the 64-bit division
    // s / SPC (a long SALU sequence per call: 15k SALU instructions a wave)
    int st_i = i_lo > 1 ? i_lo : 1, st_u = 0;
    int64_t st_s = (int64_t)(st_i - 1) * SPC;
    const int64_t s_end = (int64_t)(i_hi - 1) * SPC;  // conditioners st_i .. i_hi - 1
    auto stage_next = [&]() {
        if (st_s >= s_end) return;
        const int nblk = st_u < NH ? ((2 * st_i + 31) / 32) * NS * 2 + 1 : KBH * NS * 2 + NTG + 1;
        stage_record<kArWaves>(a.pack + 256 + (int64_t)st_s * a.sb * 256, nblk, (st_s & 1) ? slot1 : slot0, wid,
                               lane);
        ++st_s;
        if (++st_u == SPC) {
            st_u = 0;
            ++st_i;
        }
    };

    // ---- prologue: status words, the first two sub-records, the trig operands
    for (int i = threadIdx.x; i < D; i += 64 * kArWaves) cst[i] = 0;
    const float un1 = a.pack[3], un2 = a.pack[4], un3 = a.pack[5];
    h8 th[KBX], tl[KBX];  // layer-1 B operands: features 32 kb + 8 q + j of sample sl
    // the k-blocks this workgroup's conditioners read (a column range of a
    // split launch: conditioners < i_hi read features < 2 (i_hi - 1))
    const int kb_need = i_hi > 1 ? (2 * (i_hi - 1) + 31) / 32 : 0;
#pragma unroll
    for (int kb = 0; kb < KBX; ++kb) {
        th[kb] = h8{0, 0, 0, 0, 0, 0, 0, 0};
        tl[kb] = th[kb];
        if constexpr (!INV) {
            if (kb < kb_need && kb < a.kb1m) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int col = 16 * kb + 4 * q + t;
                    const float v = col < D ? a.x[brow * a.ldx + col] : 0.0f;
                    _Float16 ch, cl, sh, s2;
                    trig_split(v, a.pi, a.bnd, ch, cl, sh, s2);
                    th[kb][2 * t] = ch;
                    th[kb][2 * t + 1] = sh;
                    tl[kb][2 * t] = cl;
                    tl[kb][2 * t + 1] = s2;
                }
            }
        }
    }
    stage_next();
    stage_next();
    dma_barrier();

    int64_t s = (int64_t)(st_i - 1) * SPC;  // the sub-record the next GEMM reads
    auto slot = [&]() -> const float4* { return (s & 1) ? slot1 : slot0; };
    auto end = [&]() {
        gemm_fence();
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        stage_next();  // sub-record s + 2
#ifdef NFK_AR_DIAG_SYNC  // diagnostic: every copy waited for at once (no copy in flight during a GEMM)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
#endif
        ++s;
    };
    const float c21 = -2.0f * kL2E * un1, c22 = -2.0f * kL2E * un2;
    float ld_acc = 0.0f;  // lane group 0: this sample's log|det|, summed in column order
    float xin = 0.0f;     // spline input of this lane's column in the current pass
    h8 bh[KBH], bl[KBH];
    h4 btail = h4{0, 0, 0, 0};

    for (int i = i_lo; i < i_hi; ++i) {
        const int c = INV ? 0 : ((i - i_lo) % G);  // slab of column i
        if (c == 0) {  // first column of a pass: this lane's spline input, loaded early
            const int col = INV ? i : i + (q < G ? q : 0);
            xin = col < D ? a.x[brow * a.ldx + col] : 0.0f;
        }
        float* const slab = scr + c * 16 * PS;
        if (i == 0) {
            // coordinate 0: init_param (flows.py:178-180), the same logits for every sample
            for (int e = lane; e < 16 * P; e += 64) {
                const int r = e / P;
                slab[r * PS + (e - r * P)] = a.pack[8 + (e - r * P)];
            }
        } else {
            const int kb1 = (2 * i + 31) >> 5;
            f32x4 h[HT];
            // layer 1 on the trig operands of columns < i: the k-block past
            // feature 2i is masked (its weights are zero; the mask keeps a
            // non-finite later column out, as the reference's x[:, :i] does)
            auto layer1 = [&](auto kbc) {
                constexpr int KB = decltype(kbc)::value;
                h8 mh[KB], ml[KB];
#pragma unroll
                for (int kb = 0; kb < KB; ++kb) mh[kb] = th[kb], ml[kb] = tl[kb];
                if constexpr (!INV) {
                    const int lim = 2 * i - 32 * (KB - 1) - 8 * q;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        mh[KB - 1][j] = j < lim ? mh[KB - 1][j] : (_Float16)0.0f;
                        ml[KB - 1][j] = j < lim ? ml[KB - 1][j] : (_Float16)0.0f;
                    }
                }
                ar_parts<NS, KB, false, HT, 0>(mh, ml, btail, lane, h, slot, end, 1.0f, busy);
            };
            switch (kb1) {
                case 1: layer1(std::integral_constant<int, 1>{}); break;
                case 2: if constexpr (KBX >= 2) layer1(std::integral_constant<int, 2>{}); break;
                case 3: if constexpr (KBX >= 3) layer1(std::integral_constant<int, 3>{}); break;
                case 4: if constexpr (KBX >= 4) layer1(std::integral_constant<int, 4>{}); break;
                case 5: if constexpr (KBX >= 5) layer1(std::integral_constant<int, 5>{}); break;
                case 6: if constexpr (KBX >= 6) layer1(std::integral_constant<int, 6>{}); break;
                case 7: if constexpr (KBX >= 7) layer1(std::integral_constant<int, 7>{}); break;
                case 8: if constexpr (KBX >= 8) layer1(std::integral_constant<int, 8>{}); break;
                case 9: if constexpr (KBX >= 9) layer1(std::integral_constant<int, 9>{}); break;
                case 10: if constexpr (KBX >= 10) layer1(std::integral_constant<int, 10>{}); break;
                case 11: if constexpr (KBX >= 11) layer1(std::integral_constant<int, 11>{}); break;
                default: break;
            }
            f32x4 o[NO];
            if constexpr (TK == 2) {
                h8 b1, b2;
                act_operands16<KBH, HT>(h, c21, bh, bl, b1, b2);
                {
                    f32x4 h2[HT];
                    ar_parts16<NS, KBH, HT, 0>(bh, bl, b1, b2, lane, h2, slot, end, busy);
                    act_operands16<KBH, HT>(h2, c22, bh, bl, b1, b2);
                }
                ar_parts16<NS, KBH, NO, 0>(bh, bl, b1, b2, lane, o, slot, end, busy);
            } else {
                act_operands<KBH, T1, HT>(h, c21, bh, bl, btail);
#ifdef NFK_AR_DIAG_DUMP
                if (i == 1 && blockIdx.x == 0) ar_dump_act<HT>(0, h, KBH, wid * 16 + sl, q);
#endif
                {
                    f32x4 h2[HT];
                    ar_parts<NS, KBH, T1, HT, 0>(bh, bl, btail, lane, h2, slot, end, 1.0f, busy);
                    act_operands<KBH, T1, HT>(h2, c22, bh, bl, btail);
#ifdef NFK_AR_DIAG_DUMP
                    if (i == 1 && blockIdx.x == 0) ar_dump_act<HT>(1, h2, KBH, wid * 16 + sl, q);
#endif
                }
                ar_parts<NS, KBH, T1, NO, 0>(bh, bl, btail, lane, o, slot, end, 1.0f, busy);
            }
            // logits (unscaled: the exact power of two) into the slab, [sample][param]
#ifdef NFK_AR_DIAG_DUMP
            if (i == 1 && blockIdx.x == 0)
                for (int t = 0; t < NO; ++t)
                    for (int r = 0; r < 4; ++r) g_ar_dbg[(2 * 64 + wid * 16 + sl) * 512 + 16 * t + 4 * q + r] = o[t][r] * un3;
#endif
#pragma unroll
            for (int t = 0; t < NO; ++t) {
                const int p = 16 * t + 4 * q;
                if (p < PS - 3)
                    *reinterpret_cast<float4*>(slab + sl * PS + p) =
                        make_float4(o[t][0] * un3, o[t][1] * un3, o[t][2] * un3, o[t][3] * un3);
            }
        }
        if (!(INV || c == G - 1 || i == i_hi - 1)) continue;

        // ---- spline pass: columns i - c .. i (forward: lane group q takes
        // column i - c + q; inverse: every lane group column i)
        const int cl = INV ? 0 : (q < G ? q : 0);
        const int col = INV ? i : i - c + q;
        const bool act = INV || q <= c;  // (q <= c < G)
        float wr[K], hr[K], dr[K - 1 > 0 ? K - 1 : 1];
        {
            const float* row = scr + cl * 16 * PS + sl * PS;
#pragma unroll
            for (int p = 0; p < K; ++p) wr[p] = row[p];
#pragma unroll
            for (int p = 0; p < K; ++p) hr[p] = row[K + p];
#pragma unroll
            for (int p = 0; p < K - 1; ++p) dr[p] = row[2 * K + p];
        }
        float out, lad;
        bool inside, nd;
        nfk_rqs_element_lean<K, INV>(xin, wr, hr, dr, a.c, out, lad, inside, nd);
        const bool live = act && row_ok;
        if (live && (!INV || q == 0)) a.out[(b0 + sl) * a.ldo + col] = out;
        const float lm = act ? lad : 0.0f;
        if (!INV && a.ld_cols != nullptr) {
            // split columns: each term to its column's row, summed in column
            // order by k_ar_ld_sum (the same additions as ld_acc below)
            if (live) a.ld_cols[(int64_t)col * a.batch + b0 + sl] = lad;
        } else {
#pragma unroll
            for (int g = 0; g < G; ++g) ld_acc = ld_acc + __shfl(lm, sl + 16 * g, 64);
        }
        // status bits of each column of the pass
        const uint64_t m_in = __ballot(live && inside), m_nd = __ballot(live && inside && nd);
        if (lane == 0) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int cg = i - c + g;
                if (cg > i) break;
                const int bits = (((m_in >> (16 * g)) & 0xFFFFull) ? NFK_ST_INSIDE_SEEN : 0) |
                                 (((m_nd >> (16 * g)) & 0xFFFFull) ? NFK_ST_NEG_DISC : 0);
                if (bits) atomicOr(cst + cg, bits);
            }
        }
        if constexpr (INV) {
            // the inverted coordinate joins the trig features of the next
            // conditioners: features 2i (cos) and 2i + 1 (sin)
            if (i + 1 < D) {
                _Float16 ch, clo, sh, s2;
                trig_split(out, a.pi, a.bnd, ch, clo, sh, s2);
                const int k = 2 * i, kbi = k >> 5, qq = (k >> 3) & 3, j = k & 7;
#pragma unroll
                for (int kb = 0; kb < KBX; ++kb)
#pragma unroll
                    for (int jj = 0; jj < 8; jj += 2) {
                        const bool hit = kb == kbi && q == qq && jj == j;
                        th[kb][jj] = hit ? ch : th[kb][jj];
                        th[kb][jj + 1] = hit ? sh : th[kb][jj + 1];
                        tl[kb][jj] = hit ? clo : tl[kb][jj];
                        tl[kb][jj + 1] = hit ? s2 : tl[kb][jj + 1];
                    }
            }
        }
    }

    // ---- log|det| of the layer, the status words
    if (q == 0 && row_ok && a.mode != 0 && a.ld_cols == nullptr) {
        float* ld = a.logdet + b0 + sl;
        *ld = a.mode == 2 ? *ld + ld_acc : ld_acc;
    }
    __syncthreads();
    if (a.status != nullptr) {
        for (int i = threadIdx.x; i < D; i += 64 * kArWaves) {
            const int bits = cst[i];
            if (bits != 0 && (a.status[i] & bits) != bits) atomicOr(a.status + i, bits);
        }
    }
}

// the kernels: this unit is code-generated without packed-FP32 VALU
// instructions (Makefile NOPK: DESIGN.md section 10.5's erratum); the
// one-wave-per-SIMD instances (H = 354: 512 registers) take them back
// (NFK_PK_FP32), the instances that admit two waves per SIMD (_np) do not
template <int KBH, int TK, int K, int KBX, bool INV, int NW>
__global__ __launch_bounds__(64 * NW, 1) NFK_PK_FP32 void k_fused_ar(ArArgs a) {
    static_assert(ar_min_waves(KBH) == 1, "two-wave instances: k_fused_ar_np");
    ar_layer<KBH, TK, K, KBX, INV, NW>(a);
}
template <int KBH, int TK, int K, int KBX, bool INV, int NW>
__global__ __launch_bounds__(64 * NW, 2) void k_fused_ar_np(ArArgs a) {
    ar_layer<KBH, TK, K, KBX, INV, NW>(a);
}

// log|det| of a column-split forward: the per-column terms summed in column
// order from 0 (bitwise the single-range kernel's ld_acc), then mode 1/2.
// A workgroup takes 64 rows: waves 1-15 load 256-column chunks of the
// [dim][batch] terms into one of two LDS buffers (coalesced over the rows,
// all of a chunk's loads in flight at once) while wave 0 adds the previous
// chunk of each row in column order (16-B LDS reads, row stride 260 floats:
// conflict-free); one barrier per chunk.  (One thread per row walking the
// columns had each add wait for its strided load: 0.78 ms at Polymer's 2048
// columns; one 128-column buffer filled and summed in turn: 0.23 ms.)  The
// sum itself is the dependent chain of dim additions per row.
constexpr int kLdRows = 64, kLdCols = 256, kLdStride = kLdCols + 4, kLdThreads = 1024;
constexpr int kLdPer = (kLdRows * kLdCols + kLdThreads - 64 - 1) / (kLdThreads - 64);  // loads per loader thread
constexpr size_t kLdLds = (size_t)2 * kLdRows * kLdStride * sizeof(float);

__device__ __forceinline__ void ld_load_chunk(const float* cols, float* buf, int64_t batch, int64_t r0, int nr,
                                              int c0, int nc, int t) {
    float v[kLdPer];
#pragma unroll
    for (int i = 0; i < kLdPer; ++i) {
        const int e = t + i * (kLdThreads - 64), c = e >> 6, r = e & 63;
        v[i] = (c < nc && r < nr) ? cols[(int64_t)(c0 + c) * batch + r0 + r] : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < kLdPer; ++i) {
        const int e = t + i * (kLdThreads - 64), c = e >> 6, r = e & 63;
        if (c < nc) buf[r * kLdStride + c] = v[i];
    }
}

__global__ __launch_bounds__(kLdThreads) void k_ar_ld_sum(const float* cols, float* logdet, int64_t batch, int dim,
                                                         int mode) {
    extern __shared__ __attribute__((aligned(16))) float ldt[];
    const int t = threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.x * kLdRows;
    const int nr = batch - r0 < kLdRows ? (int)(batch - r0) : kLdRows;
    const int nch = (dim + kLdCols - 1) / kLdCols;
    if (t >= 64) ld_load_chunk(cols, ldt, batch, r0, nr, 0, dim < kLdCols ? dim : kLdCols, t - 64);
    __syncthreads();
    float acc = 0.0f;
    for (int k = 0; k < nch; ++k) {
        const int c0 = k * kLdCols, nc = dim - c0 < kLdCols ? dim - c0 : kLdCols;
        if (t >= 64) {
            if (k + 1 < nch) {
                const int c1 = c0 + kLdCols;
                ld_load_chunk(cols, ldt + ((k + 1) & 1) * kLdRows * kLdStride, batch, r0, nr, c1,
                              dim - c1 < kLdCols ? dim - c1 : kLdCols, t - 64);
            }
        } else if (t < nr) {
            const float* row = ldt + (k & 1) * kLdRows * kLdStride + t * kLdStride;
            const int n4 = nc >> 2;
            for (int c = 0; c < n4; ++c) {
                const float4 v = reinterpret_cast<const float4*>(row)[c];
                acc = acc + v.x;
                acc = acc + v.y;
                acc = acc + v.z;
                acc = acc + v.w;
            }
            for (int c = 4 * n4; c < nc; ++c) acc = acc + row[c];
        }
        __syncthreads();
    }
    if (t < nr) logdet[r0 + t] = mode == 2 ? logdet[r0 + t] + acc : acc;
}

inline void launch_ld_sum(const float* cols, float* logdet, int64_t batch, int dim, int mode, hipStream_t st) {
    hipLaunchKernelGGL(k_ar_ld_sum, dim3((unsigned)((batch + kLdRows - 1) / kLdRows)), dim3(kLdThreads), kLdLds, st,
                       cols, logdet, batch, dim, mode);
}


// column ranges of a forward launch: enough workgroups for every CU
// (resident workgroups per CU: 1 for the wide conditioners, else 8 / waves),
// one range per conditioner at most; the inverse is sequential (1)
inline int ar_csplit(const ArDims& d, int dim, int64_t batch, bool inv) {
    if (inv || batch <= 0) return 1;
    static const int forced = [] {  // diagnostic: NFK_AR_CSPLIT=n forces n column ranges (A/B runs)
        const char* e = std::getenv("NFK_AR_CSPLIT");
        return e != nullptr ? std::atoi(e) : 0;
    }();
    if (forced > 0) return forced < dim ? forced : dim;
    static const int cus = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        return n;
    }();
    const int nw = ar_waves(d);
    const int64_t rb = (batch + 16 * nw - 1) / (16 * nw);
    const int64_t want = (int64_t)cus * (ar_min_waves(d.KBH) == 1 ? 1 : 8 / nw);
    if (rb >= want) return 1;
    const int64_t cs = (want + rb - 1) / rb;
    return (int)(cs < dim ? cs : dim);
}

template <int KBH, int T1, int K, int KBX>
int launch_ar(const ArArgs& a, const ArDims& d, bool inv, hipStream_t st) {
    constexpr bool wide = ar_min_waves(KBH) == 1;  // one workgroup of 4 waves per CU
    const int nw = ar_waves(d);
    size_t lds = ar_lds_bytes(d, a.dim, inv, nw);
#ifdef NFK_AR_DIAG_PAD  // diagnostic: LDS padded to 96 KiB, one workgroup (one wave per SIMD) per CU
    lds = lds < 96 * 1024 ? 96 * 1024 : lds;
#endif
    const int64_t nblk = a.csplit > 1 ? (a.rblocks * a.csplit + 7) / 8 * 8 : a.rblocks;
    const dim3 g((unsigned)nblk), b(64 * nw);
    if constexpr (wide) {
        if (inv)
            hipLaunchKernelGGL((k_fused_ar<KBH, T1, K, KBX, true, 4>), g, b, lds, st, a);
        else
            hipLaunchKernelGGL((k_fused_ar<KBH, T1, K, KBX, false, 4>), g, b, lds, st, a);
    } else if (nw == 8) {
        if (inv)
            hipLaunchKernelGGL((k_fused_ar_np<KBH, T1, K, KBX, true, 8>), g, b, lds, st, a);
        else
            hipLaunchKernelGGL((k_fused_ar_np<KBH, T1, K, KBX, false, 8>), g, b, lds, st, a);
    } else {
        if (inv)
            hipLaunchKernelGGL((k_fused_ar_np<KBH, T1, K, KBX, true, 4>), g, b, lds, st, a);
        else
            hipLaunchKernelGGL((k_fused_ar_np<KBH, T1, K, KBX, false, 4>), g, b, lds, st, a);
    }
    if (a.csplit > 1 && a.mode != 0)
        launch_ld_sum(a.ld_cols, a.logdet, a.batch, a.dim, a.mode, st);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

// ---------------------------------------------------------------------------
// NSF_CL with a wide conditioner (nf/flows.py:216-253 at the applications'
// setup.py:59-62 sizes: hidden 354, nsplines 32), the NSF_AR machinery reused:
// ONE conditioner FCNN(n_lo, n_up (3K-1), H) per layer, so layers 1 and 2 run
// once per sample and the output layer streams as n_up records of NO tiles
// (row j (3K-1) + p = parameter p of upper coordinate j, the reshape of
// flows.py:231), each followed by its coordinate's spline (G per pass).  The
// layer-1 B operands are the sample's lower coordinates, scaled per sample by
// a power of two before the fp16 split (the bias scaled to match, the tanh
// constant unscaled per lane), as in the other fused NSF kernels.  Both
// directions share the structure (the upper coordinates do not condition each
// other); lower columns pass through.  One status word per layer.
// Pack: the AR header block, layer 1 (NH sub-records over KB1 = ceil(n_lo/32)
// k-blocks), layer 2 (NH), then n_up x N3 output sub-records, each SB blocks.
constexpr int kClKB1Max = 4;  // n_lo <= 128
__host__ __device__ inline ArDims cl_dims(int hidden, int K, int n_lo) { return ar_dims(hidden, K, 16 * ((n_lo + 31) / 32) + 1); }
__host__ __device__ inline int64_t cl_nsub(const ArDims& d, int n_up) { return 2 * (int64_t)d.NH + (int64_t)n_up * d.N3; }
__host__ __device__ inline int64_t cl_pack_floats(const ArDims& d, int n_up) { return 256 + cl_nsub(d, n_up) * d.SB * 256; }

// instantiated shapes (KBH, T1, K): the applications' H = 354, K = 32
// (Einstein / LJ / Fe_*.yaml) and config.py's defaults H = 100, K = 32
#define NFK_CL_SHAPES(X) X(11, 1, 32) X(3, 1, 32)

inline bool cl_instance(const ArDims& d, int K) {
#define NFK_CL_CHK(h, t, k) \
    if (d.KBH == h && d.T1 == t && K == k) return true;
    NFK_CL_SHAPES(NFK_CL_CHK)
#undef NFK_CL_CHK
    return false;
}

inline bool cl_ok(int n_lo, int n_up, int hidden, int K) {
    if (n_lo < 1 || n_lo > 32 * kClKB1Max || n_up < 1 || hidden < 1 || K < 2) return false;
    const ArDims d = cl_dims(hidden, K, n_lo);
    if (!cl_instance(d, K)) return false;
    return ar_lds_bytes(d, 2, false, 4) <= (size_t)kLdsBytes;
}

struct ClPackArgs {
    const float *w0, *b0, *w2, *b2, *w4, *b4;  // FCNN: [H][n_lo], [H], [H][H], [H], [n_up P][H], [n_up P]
    float* out;
    int n_lo, n_up, H, K, kb1;
    ArDims d;
};

__global__ __launch_bounds__(256) void k_cl_max(ClPackArgs a) {
    const int64_t n1 = (int64_t)a.H * a.n_lo, n2 = (int64_t)a.H * a.H, n3 = (int64_t)a.n_up * a.d.P * a.H;
    float m1 = 0.0f, m2 = 0.0f, m3 = 0.0f;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n1 + n2 + n3;
         g += (int64_t)gridDim.x * blockDim.x) {
        if (g < n1)
            m1 = fmaxf(m1, fabsf(a.w0[g]));
        else if (g < n1 + n2)
            m2 = fmaxf(m2, fabsf(a.w2[g - n1]));
        else
            m3 = fmaxf(m3, fabsf(a.w4[g - n1 - n2]));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        m1 = fmaxf(m1, __shfl_xor(m1, off, 64));
        m2 = fmaxf(m2, __shfl_xor(m2, off, 64));
        m3 = fmaxf(m3, __shfl_xor(m3, off, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        unsigned int* h = reinterpret_cast<unsigned int*>(a.out);
        atomicMax(h, __float_as_uint(m1));
        atomicMax(h + 1, __float_as_uint(m2));
        atomicMax(h + 2, __float_as_uint(m3));
    }
}

__global__ __launch_bounds__(256) void k_cl_pack(ClPackArgs a) {
    const ArDims& d = a.d;
    uint32_t* out = reinterpret_cast<uint32_t*>(a.out);
    const unsigned int* hdr = reinterpret_cast<const unsigned int*>(a.out);
    const int s1 = ar_scale_exp(__uint_as_float(hdr[0])), s2 = ar_scale_exp(__uint_as_float(hdr[1])),
              s3 = ar_scale_exp(__uint_as_float(hdr[2]));
    const int64_t total = cl_pack_floats(d, a.n_up);
    const int H = a.H, kbh = d.KBH, P = d.P, n_lo = a.n_lo;
    auto hid = [&](int t, int r) { return (d.T1 == 2 && t == 2 * kbh) ? 32 * kbh + r : hid_feature(t, r, kbh); };
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        if (g < 256) {
            if (g == 3) out[g] = __float_as_uint(ldexpf(1.0f, -(s1 + 14)));
            else if (g == 4) out[g] = __float_as_uint(ldexpf(1.0f, -(s2 + 14)));
            else if (g == 5) out[g] = __float_as_uint(ldexpf(1.0f, -(s3 + 14)));
            else if (g >= 6) out[g] = 0u;
            continue;
        }
        const int64_t w = g - 256;
        const int64_t s = w / ((int64_t)d.SB * 256);
        const int blk = (int)((w >> 8) - s * d.SB), wl = (int)(w & 255);
        uint32_t v;
        if (s < d.NH) {  // layer 1: Linear(n_lo, H) on the lower coordinates in lo_in order
            v = ar_sub_word(
                d.NS, blk, wl, a.kb1, 0, d.HT, d.NS * (int)s, ldexpf(1.0f, s1), ldexpf(1.0f, s1 + 14),
                [&](int t, int r, int k) -> float {
                    const int f = hid(t, r);
                    return (f < H && k < n_lo) ? a.w0[(int64_t)f * n_lo + k] : 0.0f;
                },
                [&](int t, int r) -> float {
                    const int f = hid(t, r);
                    return f < H ? a.b0[f] : 0.0f;
                });
        } else if (s < 2 * d.NH) {  // layer 2: Linear(H, H)
            v = ar_sub_word(
                d.NS, blk, wl, kbh, d.T1, d.HT, d.NS * (int)(s - d.NH), ldexpf(1.0f, s2), ldexpf(1.0f, s2 + 14),
                [&](int t, int r, int k) -> float {
                    const int f = hid(t, r);
                    return (f < H && k < H) ? a.w2[(int64_t)f * H + k] : 0.0f;
                },
                [&](int t, int r) -> float {
                    const int f = hid(t, r);
                    return f < H ? a.b2[f] : 0.0f;
                });
        } else {  // output layer, coordinate j: rows j P + p of Linear(H, n_up P)
            const int64_t u = s - 2 * d.NH;
            const int j = (int)(u / d.N3), part = (int)(u - (int64_t)j * d.N3);
            const int64_t r0 = (int64_t)j * P;
            v = ar_sub_word(
                d.NS, blk, wl, kbh, d.T1, d.NO, d.NS * part, ldexpf(1.0f, s3), ldexpf(1.0f, s3 + 14),
                [&](int t, int r, int k) -> float {
                    const int p = 16 * t + r;
                    return (p < P && k < H) ? a.w4[(r0 + p) * H + k] : 0.0f;
                },
                [&](int t, int r) -> float {
                    const int p = 16 * t + r;
                    return p < P ? a.b4[r0 + p] : 0.0f;
                });
        }
        out[g] = v;
    }
}

struct ClArgs {
    const float* x;
    const float* pack;
    float* z;
    float* logdet;
    int32_t* status;  // one word or null
    const int32_t *up_in, *up_out, *lo_in, *lo_out;
    int64_t ldx, ldz, batch;
    int32_t n_lo, n_up, mode, sb, kb1;
    int32_t csplit;   // upper-coordinate ranges (1: all per workgroup)
    int64_t rblocks;  // row blocks of the batch
    float* ld_cols;   // csplit > 1: per-coordinate log|det| terms [n_up][batch] (k_ar_ld_sum)
    NfkSplineConst c;
};

template <int KBH, int TK, int K, bool INV>
__device__ __forceinline__ void cl_layer(ClArgs a) {
    static_assert(TK != 2, "16-feature tails: not instanced for NSF_CL");
    constexpr int NW = 4;
    constexpr bool T1 = TK == 1;
    constexpr int HT = 2 * KBH + (TK ? 1 : 0), P = 3 * K - 1, NO = (P + 15) / 16;
    constexpr int NS = ar_ns_for(KBH);
    constexpr int NH = (HT + NS - 1) / NS, N3 = (NO + NS - 1) / NS;
    constexpr int NTG = TK == 1 ? (NS + 1) / 2 : 0;
    constexpr int PS = 16 * NO + 4, G = ar_group(false, PS);  // the upper coordinates are independent
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4, sl = lane & 15;
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    float4* const slot0 = lds4;
    float4* const slot1 = lds4 + a.sb * 64;
    float* const scr = reinterpret_cast<float*>(lds4 + 2 * a.sb * 64) + wid * (G * 16 * PS);
    int* const cst = reinterpret_cast<int*>(reinterpret_cast<float*>(lds4 + 2 * a.sb * 64) + NW * G * 16 * PS);
    // upper-coordinate range of this workgroup (a small batch splits them over
    // workgroups; XCD-affine virtual ids as in k_fused_ar)
    int sp = 0;
    int64_t rbk = blockIdx.x;
    if (a.csplit > 1) {
        const int64_t v = (int64_t)(blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
        if (v >= a.rblocks * a.csplit) return;  // padding workgroup (uniform: before any barrier)
        sp = (int)(v / a.rblocks);
        rbk = v - (int64_t)sp * a.rblocks;
    }
    const int j_lo = (int)(((int64_t)sp * a.n_up) / a.csplit), j_hi = (int)(((int64_t)(sp + 1) * a.n_up) / a.csplit);
    const int64_t b0 = (rbk * NW + wid) * 16;
    const bool row_ok = b0 + sl < a.batch;
    const bool busy = b0 < a.batch;  // (wave-uniform) any row of this wave in the batch
    const int64_t brow = row_ok ? b0 + sl : a.batch - 1;

    // the stream: layers 1 and 2 (2 NH sub-records), then the output records
    // of coordinates j_lo .. j_hi - 1; st_s counts sub-records in stream order
    const int64_t nsr = 2 * NH + (int64_t)(j_hi - j_lo) * N3;
    int64_t st_s = 0;
    auto stage_next = [&]() {
        if (st_s >= nsr) return;
        const int64_t ps = st_s < 2 * NH ? st_s : st_s + (int64_t)j_lo * N3;
        const int nblk = ps < NH ? a.kb1 * NS * 2 + 1 : KBH * NS * 2 + NTG + 1;
        stage_record<NW>(a.pack + 256 + ps * a.sb * 256, nblk, (st_s & 1) ? slot1 : slot0, wid, lane);
        ++st_s;
    };

    // ---- prologue: the status word, the lower coordinates (pass-through and
    // the layer-1 operands, scaled per sample), the first two sub-records
    if (threadIdx.x == 0) cst[0] = 0;
    const float un1 = a.pack[3], un2 = a.pack[4], un3 = a.pack[5];
    h8 xh[kClKB1Max], xl[kClKB1Max];
    float c21, bsc1;
    {
        float v[kClKB1Max][8];
        float mx = 0.0f;
#pragma unroll
        for (int kb = 0; kb < kClKB1Max; ++kb)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = 32 * kb + 8 * q + j;
                const bool ok = kb < a.kb1 && k < a.n_lo;
                const float xv = ok ? a.x[brow * a.ldx + a.lo_in[ok ? k : 0]] : 0.0f;
                v[kb][j] = xv;
                mx = fmaxf(mx, fabsf(xv));
                if (ok && row_ok && sp == 0) a.z[(b0 + sl) * a.ldz + a.lo_out[k]] = xv;  // flows.py:229-230
            }
        // per sample: the 4 lanes l, l ^ 16, l ^ 32, l ^ 48 hold one sample
        for (int off = 16; off < 64; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
        int ex = 0;
        if (mx > 0.0f && mx < 3.0e38f) frexpf(mx, &ex);
        ex = ex < -64 ? -64 : ex;  // (a tiny sample: its bias scale stays finite)
        const float sx = ldexpf(1.0f, 14 - ex);
        bsc1 = ldexpf(1.0f, -ex);
        c21 = -2.0f * kL2E * un1 * ldexpf(1.0f, ex);
#pragma unroll
        for (int kb = 0; kb < kClKB1Max; ++kb)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float t = v[kb][j] * sx;
                const _Float16 hh = (_Float16)t;
                xh[kb][j] = hh;
                xl[kb][j] = (_Float16)(t - (float)hh);
            }
    }
    stage_next();
    stage_next();
    dma_barrier();

    int64_t s = 0;
    auto slot = [&]() -> const float4* { return (s & 1) ? slot1 : slot0; };
    auto end = [&]() {
        gemm_fence();
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        stage_next();
        ++s;
    };
    const float c22 = -2.0f * kL2E * un2;
    h8 bh[KBH], bl[KBH];
    h4 btail = h4{0, 0, 0, 0};
    {
        f32x4 h[HT];
        auto layer1 = [&](auto kbc) {
            constexpr int KB = decltype(kbc)::value;
            h8 mh[KB], ml[KB];
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) mh[kb] = xh[kb], ml[kb] = xl[kb];
            ar_parts<NS, KB, false, HT, 0>(mh, ml, btail, lane, h, slot, end, bsc1, busy);
        };
        switch (a.kb1) {
            case 1: layer1(std::integral_constant<int, 1>{}); break;
            case 2: layer1(std::integral_constant<int, 2>{}); break;
            case 3: layer1(std::integral_constant<int, 3>{}); break;
            default: layer1(std::integral_constant<int, 4>{}); break;
        }
        act_operands<KBH, T1, HT>(h, c21, bh, bl, btail);
    }
    {
        f32x4 h2[HT];
        ar_parts<NS, KBH, T1, HT, 0>(bh, bl, btail, lane, h2, slot, end, 1.0f, busy);
        act_operands<KBH, T1, HT>(h2, c22, bh, bl, btail);
    }

    // ---- the upper coordinates: output record j, then the spline pass of
    // coordinates j - c .. j (lane group q takes coordinate j - c + q)
    float ld_acc = 0.0f, xin = 0.0f;
    bool any_in = false, any_nd = false;
    for (int j = j_lo; j < j_hi; ++j) {
        const int c = (j - j_lo) % G;
        if (c == 0) {
            const int col = j + (q < G ? q : 0);
            xin = col < a.n_up ? a.x[brow * a.ldx + a.up_in[col]] : 0.0f;
        }
        float* const slab = scr + c * 16 * PS;
        {
            f32x4 o[NO];
            ar_parts<NS, KBH, T1, NO, 0>(bh, bl, btail, lane, o, slot, end, 1.0f, busy);
#pragma unroll
            for (int t = 0; t < NO; ++t) {
                const int p = 16 * t + 4 * q;
                if (p < PS - 3)
                    *reinterpret_cast<float4*>(slab + sl * PS + p) =
                        make_float4(o[t][0] * un3, o[t][1] * un3, o[t][2] * un3, o[t][3] * un3);
            }
        }
        if (!(c == G - 1 || j == j_hi - 1)) continue;
        const int cl = q < G ? q : 0;
        const int col = j - c + q;
        const bool act = q <= c;
        float wr[K], hr[K], dr[K - 1 > 0 ? K - 1 : 1];
        {
            const float* row = scr + cl * 16 * PS + sl * PS;
#pragma unroll
            for (int p = 0; p < K; ++p) wr[p] = row[p];
#pragma unroll
            for (int p = 0; p < K; ++p) hr[p] = row[K + p];
#pragma unroll
            for (int p = 0; p < K - 1; ++p) dr[p] = row[2 * K + p];
        }
        float out, lad;
        bool inside, nd;
        nfk_rqs_element_lean<K, INV>(xin, wr, hr, dr, a.c, out, lad, inside, nd);
        const bool live = act && row_ok;
        if (live) a.z[(b0 + sl) * a.ldz + a.up_out[col]] = out;
        const float lm = act ? lad : 0.0f;
        if (a.ld_cols != nullptr) {
            // split coordinates: each term to its coordinate's row, summed in
            // coordinate order by k_ar_ld_sum (the additions of ld_acc below)
            if (live) a.ld_cols[(int64_t)col * a.batch + b0 + sl] = lad;
        } else {
#pragma unroll
            for (int g = 0; g < G; ++g) ld_acc = ld_acc + __shfl(lm, sl + 16 * g, 64);
        }
        any_in |= live && inside;
        any_nd |= live && inside && nd;
    }

    // ---- log|det| of the layer (flows.py:238, 252), the status word
    if (q == 0 && row_ok && a.mode != 0 && a.ld_cols == nullptr) {
        float* ld = a.logdet + b0 + sl;
        *ld = a.mode == 2 ? *ld + ld_acc : ld_acc;
    }
    const int bits = (__any(any_in) ? NFK_ST_INSIDE_SEEN : 0) | (__any(any_nd) ? NFK_ST_NEG_DISC : 0);
    if (lane == 0 && bits != 0) atomicOr(cst, bits);
    __syncthreads();
    if (a.status != nullptr && threadIdx.x == 0) {
        const int b = cst[0];
        if (b != 0 && (a.status[0] & b) != b) atomicOr(a.status, b);
    }
}
// the kernels: this unit is code-generated without packed-FP32 VALU
// instructions (Makefile NOPK: DESIGN.md section 10.5's erratum); the
// one-wave-per-SIMD instances (H = 354: 512 registers) take them back
// (NFK_PK_FP32), the instances that admit two waves per SIMD (_np) do not
template <int KBH, int TK, int K, bool INV>
__global__ __launch_bounds__(256, 1) NFK_PK_FP32 void k_fused_cl(ClArgs a) {
    static_assert(ar_min_waves(KBH) == 1, "two-wave instances: k_fused_cl_np");
    cl_layer<KBH, TK, K, INV>(a);
}
template <int KBH, int TK, int K, bool INV>
__global__ __launch_bounds__(256, 1) void k_fused_cl_np(ClArgs a) {
    cl_layer<KBH, TK, K, INV>(a);
}

// upper-coordinate ranges of a launch: enough workgroups for every CU (one
// 4-wave workgroup per CU), at most one range per coordinate
inline int cl_csplit(int n_up, int64_t batch) {
    static const int cus = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        return n;
    }();
    if (batch <= 0) return 1;
    const int64_t rb = (batch + 63) / 64;
    if (rb >= cus) return 1;
    const int64_t cs = (cus + rb - 1) / rb;
    return (int)(cs < n_up ? cs : n_up);
}

template <int KBH, int T1, int K>
int launch_cl(const ClArgs& a, const ArDims& d, bool inv, hipStream_t st) {
    const size_t lds = ar_lds_bytes(d, 2, false, 4);
    const int64_t nblk = a.csplit > 1 ? (a.rblocks * a.csplit + 7) / 8 * 8 : a.rblocks;
    const dim3 g((unsigned)nblk), b(256);
    if constexpr (ar_min_waves(KBH) == 1) {
        if (inv)
            hipLaunchKernelGGL((k_fused_cl<KBH, T1, K, true>), g, b, lds, st, a);
        else
            hipLaunchKernelGGL((k_fused_cl<KBH, T1, K, false>), g, b, lds, st, a);
    } else {
        if (inv)
            hipLaunchKernelGGL((k_fused_cl_np<KBH, T1, K, true>), g, b, lds, st, a);
        else
            hipLaunchKernelGGL((k_fused_cl_np<KBH, T1, K, false>), g, b, lds, st, a);
    }
    if (a.csplit > 1 && a.mode != 0)
        launch_ld_sum(a.ld_cols, a.logdet, a.batch, a.n_up, a.mode, st);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}


// ---------------------------------------------------------------------------
// NSF_AR with STREAMED layer-1 operands (k_fused_ar_s, forward): the wide
// layers the register instances above cannot hold -- Polymer.yaml's 2048
// coordinates (applications/input/Polymer.yaml:8-9: 2,047 conditioners
// FCNN(2i, 95, 100), flows.py:165-166, 0.42 G weights per layer).  Conditioner
// i's layer 1 reads ceil(2i / 32) k-blocks of trig features (up to 128): they
// are not kept in registers but computed once per launch into a workspace
// (k_ars_trig, in the MFMA B-operand lane layout, fp16 hi/lo of 2^14 x
// cos / sin) and streamed through the LDS slots with the weights, two k-blocks
// per sub-record (layer 1 in k-block-major order: every hidden tile of the
// k-blocks, then their trig operands for the workgroup's four waves), so each
// accumulator sees the same products in the same order as the register form
// (gemm_h: per k-block lo.hi, hi.lo, hi.hi).  Layers 2 and 3 and the spline
// are the register form's.  Given x the conditioners are independent
// (flows.py:182-189), so the launch splits them over workgroups: conditioner
// pairs (p, dim - p), whose layer-1 sizes sum to a constant, in contiguous
// ranges (balanced weight streams), the XCD-affine grid of the column split;
// every weight byte is read from HBM once per row block.  Per-column log|det|
// terms go to the workspace and k_ar_ld_sum adds them in column order
// (bitwise any partition).  The inverse is sequential through the outputs
// and stays on the per-column path.
#ifndef NFK_ARS_KBS
#define NFK_ARS_KBS 2
#endif
#ifndef NFK_ARS_NSL
#define NFK_ARS_NSL 2
#endif
constexpr int kArsKBS = NFK_ARS_KBS;  // layer-1 k-blocks per sub-record
// LDS slots of the sub-record ring: the copy of sub-record s + NSL is issued
// at the barrier that ends s, and the wait before s + 1 counts only the copies
// issued after s + 1's (vmcnt(n)), so NSL - 1 copies are in flight per GEMM
constexpr int kArsNSL = NFK_ARS_NSL;
constexpr int kArsNW = 4;   // waves per workgroup (16 rows each)

struct ArsDims {
    ArDims d;
    int SB2;  // blocks of a layer-2 / output sub-record (the register form's)
    int TB0;  // first trig block of a layer-1 sub-record in the slot
    int SBS;  // slot blocks
    int KB1M;
};

__host__ __device__ inline ArsDims ars_dims(int hidden, int K, int dim) {
    ArsDims a{};
    a.d = ar_dims(hidden, K, dim);
    a.SB2 = a.d.KBH * a.d.NS * 2 + a.d.NTG + 1;
    a.TB0 = 1 + kArsKBS * a.d.HT * 2;
    const int s1 = a.TB0 + kArsKBS * kArsNW * 2;
    a.SBS = s1 > a.SB2 ? s1 : a.SB2;
    a.KB1M = a.d.KB1M;
    return a;
}
// sum_{j=1}^{m} ceil(j / 16): layer-1 k-blocks of conditioners 1 .. m
__host__ __device__ inline int64_t ars_kb_sum(int m) {
    const int64_t q = m / 16, r = m % 16;
    return 16 * q * (q + 1) / 2 + r * (q + 1);
}
__host__ __device__ inline int ars_kb1(int i) { return (2 * i + 31) / 32; }
// pack block of conditioner i's stream (block 0 = the header): its bias block,
// kb1(i) x HT x {hi, lo} layer-1 blocks, then NH + N3 sub-records of SB2 blocks
__host__ __device__ inline int64_t ars_cond_off(const ArsDims& a, int i) {
    return 1 + (int64_t)(i - 1) * (1 + (int64_t)(a.d.NH + a.d.N3) * a.SB2) + (int64_t)a.d.HT * 2 * ars_kb_sum(i - 1);
}
__host__ __device__ inline int64_t ars_pack_floats(const ArsDims& a, int dim) { return ars_cond_off(a, dim) * 256; }
inline int64_t ars_trig_floats(const ArsDims& a, int64_t rblocks) { return rblocks * a.KB1M * kArsNW * 2 * 256; }
__host__ __device__ constexpr int ars_group(int ps) { return ps <= 52 ? 4 : 2; }
inline size_t ars_lds_bytes(const ArsDims& a, int dim) {
    return (size_t)kArsNSL * a.SBS * 1024 + (size_t)kArsNW * ars_group(a.d.PS) * 16 * a.d.PS * sizeof(float) +
           (size_t)(dim + 3) / 4 * 16;
}

// instantiated (KBH, T1, K): Polymer.yaml's conditioners (config.py:40's
// hidden 100, nsplines 32)
#define NFK_ARS_SHAPES(X) X(3, 1, 32)

inline bool ars_ok(int dim, int hidden, int K) {
    if (dim < 2 || dim > 16384 || hidden < 1 || K < 2) return false;
    const ArsDims a = ars_dims(hidden, K, dim);
    bool inst = false;
#define NFK_ARS_CHK(h, t, k) inst |= (a.d.KBH == h && a.d.T1 == t && K == k);
    NFK_ARS_SHAPES(NFK_ARS_CHK)
#undef NFK_ARS_CHK
    return inst && ars_lds_bytes(a, dim) <= (size_t)kLdsBytes;
}

__global__ __launch_bounds__(256) void k_ars_pack(ArPackArgs a) {
    const ArsDims A = ars_dims(a.H, a.K, a.dim);
    const ArDims& d = A.d;
    const int i = 1 + (int)blockIdx.y;  // conditioner
    uint32_t* out = reinterpret_cast<uint32_t*>(a.out);
    const unsigned int* hdr = reinterpret_cast<const unsigned int*>(a.out);
    const int s1 = ar_scale_exp(__uint_as_float(hdr[0])), s2 = ar_scale_exp(__uint_as_float(hdr[1])),
              s3 = ar_scale_exp(__uint_as_float(hdr[2]));
    if (i == 1 && blockIdx.x == 0) {  // the header block
        for (int g = threadIdx.x; g < 256; g += blockDim.x) {
            if (g == 3) out[g] = __float_as_uint(ldexpf(1.0f, -(s1 + 14)));
            else if (g == 4) out[g] = __float_as_uint(ldexpf(1.0f, -(s2 + 14)));
            else if (g == 5) out[g] = __float_as_uint(ldexpf(1.0f, -(s3 + 14)));
            else if (g >= 8 && g < 8 + d.P) out[g] = __float_as_uint(a.init[g - 8]);
            else if (g >= 6) out[g] = 0u;
        }
    }
    const int H = a.H, kbh = d.KBH, HT = d.HT, kb1 = ars_kb1(i);
    const float* const* pw = a.w + (int64_t)(i - 1) * 6;
    const float *W1 = pw[0], *b1 = pw[1], *W2 = pw[2], *b2 = pw[3], *W3 = pw[4], *b3 = pw[5];
    auto hid = [&](int t, int r) { return (d.T1 == 2 && t == 2 * kbh) ? 32 * kbh + r : hid_feature(t, r, kbh); };
    const int64_t base = ars_cond_off(A, i) * 256;
    const int64_t l1w = (int64_t)(1 + kb1 * HT * 2) * 256;
    const int64_t nw = l1w + (int64_t)(d.NH + d.N3) * A.SB2 * 256;
    const float sc1 = ldexpf(1.0f, s1), bsc1 = ldexpf(1.0f, s1 + 14);
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
        const int blk = (int)(w >> 8), wl = (int)(w & 255);
        uint32_t v;
        if (blk == 0) {  // layer-1 bias block [tile][row]
            const int tt = wl >> 4, r = wl & 15;
            const int f = tt < HT ? hid(tt, r) : H;
            v = __float_as_uint(f < H ? b1[f] * bsc1 : 0.0f);
        } else if (w < l1w) {  // layer 1, k-block-major: (kb, tile, {hi, lo}), canonical trig order
            const int e = blk - 1, part = e & 1, t = (e >> 1) % HT, kb = (e >> 1) / HT;
            const int lane = wl >> 2, j = 2 * (wl & 3), k0 = 32 * kb + 8 * (lane >> 4) + j, f = hid(t, lane & 15);
            auto val = [&](int k) -> float {
                if (f >= H || k >= 2 * i) return 0.0f;
                return W1[(int64_t)f * 2 * i + (k & 1) * i + (k >> 1)] * sc1;  // cat(cos, sin) columns
            };
            v = nfk_f16_part_pair(val(k0), val(k0 + 1), part);
        } else {
            const int rel = (int)((w - l1w) >> 8), sub = rel / A.SB2, b = rel - sub * A.SB2;
            if (sub < d.NH) {  // layer 2: Linear(H, H)
                v = ar_sub_word(
                    d.NS, b, wl, kbh, d.T1, d.HT, d.NS * sub, ldexpf(1.0f, s2), ldexpf(1.0f, s2 + 14),
                    [&](int t, int r, int k) -> float {
                        const int f = hid(t, r);
                        return (f < H && k < H) ? W2[(int64_t)f * H + k] : 0.0f;
                    },
                    [&](int t, int r) -> float {
                        const int f = hid(t, r);
                        return f < H ? b2[f] : 0.0f;
                    });
            } else {  // output layer: Linear(H, 3K-1)
                const int P = d.P;
                v = ar_sub_word(
                    d.NS, b, wl, kbh, d.T1, d.NO, d.NS * (sub - d.NH), ldexpf(1.0f, s3), ldexpf(1.0f, s3 + 14),
                    [&](int t, int r, int k) -> float {
                        const int p = 16 * t + r;
                        return (p < P && k < H) ? W3[(int64_t)p * H + k] : 0.0f;
                    },
                    [&](int t, int r) -> float {
                        const int p = 16 * t + r;
                        return p < P ? b3[p] : 0.0f;
                    });
            }
        }
        out[base + w] = v;
    }
}

// the trig features of every row block in the MFMA B-operand layout: block
// ((rb KB1M + kb) NW + w) 2 + {hi, lo}, lane l = (q, sl): features
// 32 kb + 8 q + j (feature 2c = cos, 2c + 1 = sin of column c < dim - 1) of
// row (rb NW + w) 16 + sl (rows past the batch repeat the last row, as the
// register form's brow), x 2^14, fp16 hi and lo
__global__ __launch_bounds__(256) void k_ars_trig(const float* x, int64_t ldx, float* trig, int64_t batch, int dim,
                                                  int kb1m, int64_t rblocks, float pi, float bnd) {
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t nrec = rblocks * kb1m * kArsNW;
    if (g >= nrec * 64) return;
    const int lane = (int)(g & 63);
    const int64_t rec = g >> 6;  // (rb, kb, w)
    const int w = (int)(rec % kArsNW), kb = (int)((rec / kArsNW) % kb1m);
    const int64_t rb = rec / ((int64_t)kArsNW * kb1m);
    const int q = lane >> 4, sl = lane & 15;
    int64_t row = (rb * kArsNW + w) * 16 + sl;
    row = row < batch ? row : batch - 1;
    h8 hi, lo;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int col = 16 * kb + 4 * q + t;
        _Float16 ch = 0, cl = 0, sh = 0, s2 = 0;
        if (col < dim - 1) trig_split(x[row * ldx + col], pi, bnd, ch, cl, sh, s2);
        hi[2 * t] = ch;
        hi[2 * t + 1] = sh;
        lo[2 * t] = cl;
        lo[2 * t + 1] = s2;
    }
    float4* dst = reinterpret_cast<float4*>(trig + rec * 2 * 256);
    dst[lane] = __builtin_bit_cast(float4, hi);
    dst[64 + lane] = __builtin_bit_cast(float4, lo);
}

struct ArsArgs {
    const float* x;
    const float* pack;
    const float* trig;
    float* out;
    float* ld_cols;   // [dim][batch] per-column log|det| terms
    int32_t* status;  // [dim] or null
    int64_t ldx, ldo, batch, rblocks;
    int32_t dim, sbs, kb1m, csplit, npair;
    NfkSplineConst c;
};

template <int KBH, int TK, int K>
__global__ __launch_bounds__(64 * kArsNW, 1) void k_fused_ar_s(ArsArgs a) {
    constexpr int NW = kArsNW;
    constexpr bool T1 = TK == 1;
    static_assert(TK != 2, "16-feature tails: not instanced for the streamed form");
    constexpr int HT = 2 * KBH + (TK ? 1 : 0), P = 3 * K - 1, NO = (P + 15) / 16;
    constexpr int NS = ar_ns_for(KBH);
    constexpr int NH = (HT + NS - 1) / NS, N3 = (NO + NS - 1) / NS;
    constexpr int NTG = TK == 1 ? (NS + 1) / 2 : 0;
    constexpr int SB2 = KBH * NS * 2 + NTG + 1;
    constexpr int TB0 = 1 + kArsKBS * HT * 2;
    constexpr int PS = 16 * NO + 4, G = ars_group(PS);
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4, sl = lane & 15;
    const int D = a.dim;
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    auto slot_of = [&](int n) -> float4* { return lds4 + (n % kArsNSL) * a.sbs * 64; };
    float* const scr = reinterpret_cast<float*>(lds4 + kArsNSL * a.sbs * 64) + wid * (G * 16 * PS);
    int* const cst = reinterpret_cast<int*>(reinterpret_cast<float*>(lds4 + kArsNSL * a.sbs * 64) + NW * G * 16 * PS);
    // XCD-affine grid (k_fused_ar): the row blocks of one conditioner range share an XCD
    const int64_t v = (int64_t)(blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    if (v >= a.rblocks * a.csplit) return;  // padding workgroup (uniform: before any barrier)
    const int sp = (int)(v / a.rblocks);
    const int64_t rbk = v - (int64_t)sp * a.rblocks;
    const int p_lo = 1 + (int)(((int64_t)sp * a.npair) / a.csplit), p_hi = 1 + (int)(((int64_t)(sp + 1) * a.npair) / a.csplit);
    const int64_t b0 = (rbk * NW + wid) * 16;
    const bool row_ok = b0 + sl < a.batch;
    const bool busy = b0 < a.batch;  // (wave-uniform) any row of this wave in the batch
    const int64_t brow = row_ok ? b0 + sl : a.batch - 1;
    // the conditioners of pair p: p, then dim - p (one when they coincide)
    auto cond_of = [&](int p, int m) { return m == 0 ? p : D - p; };
    auto members = [&](int p) { return D - p != p ? 2 : 1; };

    // sub-record cursor in stream order: pair st_p, member st_m, part st_u
    // (layer-1 parts 0 .. NU1 - 1, then NH layer-2 and N3 output parts)
    int st_p = p_lo, st_m = 0, st_u = 0, st_n = 0;
    // this wave's DMA instructions of the copies after the one being consumed
    // (sub-records s + 1 .. s + NSL - 1), oldest first
    static_assert(kArsNSL >= 2 && kArsNSL <= 4, "2 to 4 slots");
    int pq0 = 0, pq1 = 0, pq2 = 0;
    const ArsDims AD = ars_dims(32 * KBH + (TK == 1 ? 4 : 0), K, D);  // (only the block offsets are used)
    // issue the copy of sub-record st_n; returns this wave's DMA instructions
    // (0 past the stream's end, where nothing is issued)
    auto stage_next = [&]() -> int {
        int cnt = 0;
        if (st_p >= p_hi) return 0;
        const int i = cond_of(st_p, st_m), kb1 = ars_kb1(i), nu1 = (kb1 + kArsKBS - 1) / kArsKBS;
        float4* const dst = slot_of(st_n);
        const float* cb = a.pack + ars_cond_off(AD, i) * 256;
        const uint32_t base = lds_addr(dst);
        if (st_u < nu1) {
            const int kb0 = st_u * kArsKBS, nk = kb1 - kb0 < kArsKBS ? kb1 - kb0 : kArsKBS;
            // weights (with the bias block in front of part 0), then the trig operands
            const int wb0 = st_u == 0 ? 0 : 1, nwb = (st_u == 0 ? 1 : 0) + nk * HT * 2;
            const float* wsrc = cb + (int64_t)(st_u == 0 ? 0 : 1 + kb0 * HT * 2) * 256;
            for (int b = wid; b < nwb; b += NW) dma_blk(wsrc + (int64_t)b * 256, lane, base + (wb0 + b) * 1024);
            const float* tsrc = a.trig + ((rbk * a.kb1m + kb0) * NW) * 2 * 256;
            for (int b = wid; b < nk * NW * 2; b += NW) dma_blk(tsrc + (int64_t)b * 256, lane, base + (TB0 + b) * 1024);
            cnt = (nwb > wid ? (nwb - wid + NW - 1) / NW : 0) + (nk * NW * 2 - wid + NW - 1) / NW;
        } else {
            const int k = st_u - nu1;
            const float* src = cb + (int64_t)(1 + kb1 * HT * 2 + k * SB2) * 256;
            for (int b = wid; b < SB2; b += NW) dma_blk(src + (int64_t)b * 256, lane, base + b * 1024);
            cnt = (SB2 - wid + NW - 1) / NW;
        }
        ++st_n;
        if (++st_u == nu1 + NH + N3) {
            st_u = 0;
            if (++st_m == members(st_p)) {
                st_m = 0;
                ++st_p;
            }
        }
        return cnt;
    };

    // ---- prologue: status words, the first NSL sub-records (wait for the first)
    for (int i = threadIdx.x; i < D; i += 64 * NW) cst[i] = 0;
    const float un1 = a.pack[3], un2 = a.pack[4], un3 = a.pack[5];
    stage_next();
    pq0 = stage_next();
    if (kArsNSL > 2) pq1 = stage_next();
    if (kArsNSL > 3) pq2 = stage_next();
    {
        wait_vmcnt_le(pq0 + pq1 + pq2);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    }

    int s = 0;  // sub-records consumed
    auto slot = [&]() -> const float4* { return slot_of(s); };
    auto end = [&]() {
        gemm_fence();
        // sub-record s + 1 landed: only the copies issued after it may be in flight
        wait_vmcnt_le(pq1 + pq2);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const int c = stage_next();  // sub-record s + NSL, into the slot of s
        if (kArsNSL == 2) pq0 = c;
        if (kArsNSL == 3) pq0 = pq1, pq1 = c;
        if (kArsNSL == 4) pq0 = pq1, pq1 = pq2, pq2 = c;
        ++s;
    };
    const float c21 = -2.0f * kL2E * un1, c22 = -2.0f * kL2E * un2;
    h8 bh[KBH], bl[KBH];
    h4 btail = h4{0, 0, 0, 0};
    int cols[G];   // the slabs' columns (uniform)
    int nc = 0;    // slabs filled
    bool any = false;

    // the spline pass over the nc filled slabs: lane group g < nc takes column cols[g]
    auto spline_pass = [&]() {
        const bool act = q < nc;
        const int col = cols[q < nc ? q : 0];
        const float xin = a.x[brow * a.ldx + col];
        float wr[K], hr[K], dr[K - 1 > 0 ? K - 1 : 1];
        const float* row = scr + (q < nc ? q : 0) * 16 * PS + sl * PS;
#pragma unroll
        for (int p = 0; p < K; ++p) wr[p] = row[p];
#pragma unroll
        for (int p = 0; p < K; ++p) hr[p] = row[K + p];
#pragma unroll
        for (int p = 0; p < K - 1; ++p) dr[p] = row[2 * K + p];
        float out, lad;
        bool inside, nd;
        nfk_rqs_element_lean<K, false>(xin, wr, hr, dr, a.c, out, lad, inside, nd);
        const bool live = act && row_ok;
        if (live) {
            a.out[(b0 + sl) * a.ldo + col] = out;
            a.ld_cols[(int64_t)col * a.batch + b0 + sl] = lad;
        }
        const uint64_t m_in = __ballot(live && inside), m_nd = __ballot(live && inside && nd);
        if (lane == 0) {
            for (int g = 0; g < nc; ++g) {
                const int bits = (((m_in >> (16 * g)) & 0xFFFFull) ? NFK_ST_INSIDE_SEEN : 0) |
                                 (((m_nd >> (16 * g)) & 0xFFFFull) ? NFK_ST_NEG_DISC : 0);
                if (bits) atomicOr(cst + cols[g], bits);
            }
        }
        nc = 0;
    };

    // column 0: init_param (flows.py:178-180), by the first range
    if (sp == 0) {
        for (int e = lane; e < 16 * P; e += 64) {
            const int r = e / P;
            scr[r * PS + (e - r * P)] = a.pack[8 + (e - r * P)];
        }
        cols[0] = 0;
        nc = 1;
        any = true;
    }
    for (int p = p_lo; p < p_hi; ++p) {
        for (int m = 0; m < members(p); ++m) {
            const int i = cond_of(p, m), kb1 = ars_kb1(i);
            f32x4 h[HT];
            // ---- layer 1, k-block-major over the streamed sub-records
            for (int kb0 = 0; kb0 < kb1; kb0 += kArsKBS) {
                const float4* sl4 = slot();
                if (kb0 == 0) {
#pragma unroll
                    for (int t = 0; t < HT; ++t) h[t] = as_f32x4(sl4[t * 4 + q]);
                }
                const int nk = kb1 - kb0 < kArsKBS ? kb1 - kb0 : kArsKBS;
                for (int kl = 0; kl < (busy ? nk : 0); ++kl) {
                    h8 th = __builtin_bit_cast(h8, sl4[(TB0 + (kl * NW + wid) * 2) * 64 + lane]);
                    h8 tl = __builtin_bit_cast(h8, sl4[(TB0 + (kl * NW + wid) * 2 + 1) * 64 + lane]);
                    if (kb0 + kl == kb1 - 1) {  // the k-block past feature 2i: masked (x[:, :i])
                        const int lim = 2 * i - 32 * (kb1 - 1) - 8 * q;
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            th[j] = j < lim ? th[j] : (_Float16)0.0f;
                            tl[j] = j < lim ? tl[j] : (_Float16)0.0f;
                        }
                    }
#pragma unroll
                    for (int t = 0; t < HT; ++t) {
                        const h8 ahi = __builtin_bit_cast(h8, sl4[(1 + (kl * HT + t) * 2) * 64 + lane]);
                        const h8 alo = __builtin_bit_cast(h8, sl4[(1 + (kl * HT + t) * 2 + 1) * 64 + lane]);
                        h[t] = mfma16(alo, th, h[t]);
                        h[t] = mfma16(ahi, tl, h[t]);
                        h[t] = mfma16(ahi, th, h[t]);
                    }
                }
                mfma_result_wait();
                end();
            }
            act_operands<KBH, T1, HT>(h, c21, bh, bl, btail);
            {
                f32x4 h2[HT];
                ar_parts<NS, KBH, T1, HT, 0>(bh, bl, btail, lane, h2, slot, end, 1.0f, busy);
                act_operands<KBH, T1, HT>(h2, c22, bh, bl, btail);
            }
            f32x4 o[NO];
            ar_parts<NS, KBH, T1, NO, 0>(bh, bl, btail, lane, o, slot, end, 1.0f, busy);
            float* const slab = scr + nc * 16 * PS;
#pragma unroll
            for (int t = 0; t < NO; ++t) {
                const int pp = 16 * t + 4 * q;
                if (pp < PS - 3)
                    *reinterpret_cast<float4*>(slab + sl * PS + pp) =
                        make_float4(o[t][0] * un3, o[t][1] * un3, o[t][2] * un3, o[t][3] * un3);
            }
            cols[nc++] = i;
            any = true;
            if (nc == G) spline_pass();
        }
    }
    if (nc > 0) spline_pass();
    __syncthreads();
    if (a.status != nullptr && any) {
        for (int i = threadIdx.x; i < D; i += 64 * NW) {
            const int bits = cst[i];
            if (bits != 0 && (a.status[i] & bits) != bits) atomicOr(a.status + i, bits);
        }
    }
}

// conditioner-pair ranges of a launch: enough workgroups for every CU (one
// per CU), at most one pair each
inline int ars_csplit(int npair, int64_t rblocks) {
    static const int cus = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
        return n;
    }();
    const int64_t cs = rblocks >= cus ? 1 : (cus + rblocks - 1) / rblocks;
    return (int)(cs < npair ? cs : npair);
}

template <int KBH, int T1, int K>
int launch_ars(ArsArgs a, const ArsDims& ad, float* logdet, int mode, float pi, float bnd, hipStream_t st) {
    const int64_t ntrig = a.rblocks * a.kb1m * kArsNW * 64;
    hipLaunchKernelGGL(k_ars_trig, dim3((unsigned)((ntrig + 255) / 256)), dim3(256), 0, st, a.x, a.ldx,
                       const_cast<float*>(a.trig), a.batch, a.dim, a.kb1m, a.rblocks, pi, bnd);
    const size_t lds = ars_lds_bytes(ad, a.dim);
    const int64_t nblk = (a.rblocks * a.csplit + 7) / 8 * 8;
    hipLaunchKernelGGL((k_fused_ar_s<KBH, T1, K>), dim3((unsigned)nblk), dim3(64 * kArsNW), lds, st, a);
    if (mode != 0)
        launch_ld_sum(a.ld_cols, logdet, a.batch, a.dim, mode, st);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

}  // namespace

// the streamed form (k_fused_ar_s) for shapes beyond the register instances;
// NFK_AR_STREAM=1 or nfk_debug_ar_stream(1) (diagnostic) selects it for every
// shape it has, so it can be checked bitwise against the register form
static int g_ar_stream = -1;
static bool ar_use_stream(int dim, int hidden, int K) {
    static const bool env = [] {
        const char* e = std::getenv("NFK_AR_STREAM");
        return e != nullptr && e[0] == '1';
    }();
    if (!ars_ok(dim, hidden, K)) return false;
    const bool force = g_ar_stream < 0 ? env : g_ar_stream == 1;
    return force || !ar_ok(dim, hidden, K);
}

// Diagnostic: -1 automatic, 1 = the streamed form wherever it is instanced
// (packs built before a change must be rebuilt).  Returns the previous
// setting.  Not part of include/nfk.h.
extern "C" int nfk_debug_ar_stream(int on) {
    const int prev = g_ar_stream;
    g_ar_stream = on < 0 ? -1 : (on ? 1 : 0);
    return prev;
}

extern "C" int nfk_fused_ar_supported(int32_t dim, int32_t hidden, int32_t K) {
    return (ar_ok(dim, hidden, K) || ars_ok(dim, hidden, K)) ? 1 : 0;
}

extern "C" int nfk_fused_ar_inverse_supported(int32_t dim, int32_t hidden, int32_t K) {
    return (ar_ok(dim, hidden, K) && !ar_use_stream(dim, hidden, K)) ? 1 : 0;
}

extern "C" int64_t nfk_fused_ar_pack_elems(int32_t dim, int32_t hidden, int32_t K) {
    if (ar_use_stream(dim, hidden, K)) return ars_pack_floats(ars_dims(hidden, K, dim), dim);
    if (!ar_ok(dim, hidden, K)) return 0;
    return ar_pack_floats(ar_dims(hidden, K, dim), dim);
}

extern "C" int nfk_fused_ar_pack(const float* const* weights, const float* init_param, int32_t dim,
                                 int32_t hidden, int32_t K, float* pack, nfk_stream_t stream) {
    const bool strm = ar_use_stream(dim, hidden, K);
    if (!strm && !ar_ok(dim, hidden, K)) return nfk_set_error("nfk_fused_ar_pack: shape not supported");
    if (!weights || !init_param || !pack) return nfk_set_error("nfk_fused_ar_pack: null pointer");
    ArPackArgs a{weights, init_param, pack, dim, hidden, K, ar_dims(hidden, K, dim)};
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(pack, 0, 3 * sizeof(float), st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_ar_max, dim3(16, (unsigned)(dim - 1)), dim3(256), 0, st, a);
    if (strm) {  // conditioner by conditioner (grid y), the streamed layout
        hipLaunchKernelGGL(k_ars_pack, dim3(16, (unsigned)(dim - 1)), dim3(256), 0, st, a);
        e = hipGetLastError();
        return e == hipSuccess ? 0 : (int)e;
    }
    int64_t g = (ar_pack_floats(a.d, dim) + 255) / 256;
    if (g > 16384) g = 16384;
    hipLaunchKernelGGL(k_ar_pack, dim3((unsigned)g), dim3(256), 0, st, a);
    e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

extern "C" int64_t nfk_fused_ar_workspace(int32_t dim, int32_t hidden, int32_t K, int64_t batch, int32_t inverse) {
    if (batch <= 0) return 0;
    if (ar_use_stream(dim, hidden, K)) {
        if (inverse) return 0;
        const ArsDims ad = ars_dims(hidden, K, dim);
        return (int64_t)dim * batch + ars_trig_floats(ad, (batch + 16 * kArsNW - 1) / (16 * kArsNW));
    }
    if (!ar_ok(dim, hidden, K)) return 0;
    return ar_csplit(ar_dims(hidden, K, dim), dim, batch, inverse != 0) > 1 ? (int64_t)dim * batch : 0;
}

extern "C" int nfk_fused_ar(const float* x, int64_t ldx, const float* pack, int32_t dim, int32_t hidden, int32_t K,
                            double tail_bound, float* out, int64_t ldo, float* logdet, int32_t logdet_mode,
                            int64_t batch, int32_t inverse, int32_t* status, nfk_stream_t stream) {
    return nfk_fused_ar_ws(x, ldx, pack, dim, hidden, K, tail_bound, out, ldo, logdet, logdet_mode, batch, inverse,
                           status, nullptr, 0, stream);
}

extern "C" int nfk_fused_ar_ws(const float* x, int64_t ldx, const float* pack, int32_t dim, int32_t hidden, int32_t K,
                               double tail_bound, float* out, int64_t ldo, float* logdet, int32_t logdet_mode,
                               int64_t batch, int32_t inverse, int32_t* status, float* workspace,
                               int64_t workspace_floats, nfk_stream_t stream) {
    const bool strm = ar_use_stream(dim, hidden, K);
    if (!strm && !ar_ok(dim, hidden, K)) return nfk_set_error("nfk_fused_ar: shape not supported");
    if (batch < 0) return nfk_set_error("nfk_fused_ar: bad batch");
    if (batch == 0) return 0;
    if (!x || !pack || !out) return nfk_set_error("nfk_fused_ar: null pointer");
    if (logdet_mode != 0 && !logdet) return nfk_set_error("nfk_fused_ar: null logdet");
    if (ldx < dim || ldo < dim) return nfk_set_error("nfk_fused_ar: bad leading dimension");
    if (strm) {
        if (inverse) return nfk_set_error("nfk_fused_ar: the inverse of this shape is not fused "
                                          "(nfk_fused_ar_inverse_supported)");
        const ArsDims ad = ars_dims(hidden, K, dim);
        ArsArgs s;
        s.rblocks = (batch + 16 * kArsNW - 1) / (16 * kArsNW);
        const int64_t need = (int64_t)dim * batch + ars_trig_floats(ad, s.rblocks);
        if (workspace == nullptr || workspace_floats < need)
            return nfk_set_error("nfk_fused_ar: this shape needs nfk_fused_ar_workspace() floats of workspace");
        s.x = x;
        s.pack = pack;
        s.ld_cols = workspace;
        s.trig = workspace + (int64_t)dim * batch;
        s.out = out;
        s.status = status;
        s.ldx = ldx;
        s.ldo = ldo;
        s.batch = batch;
        s.dim = dim;
        s.sbs = ad.SBS;
        s.kb1m = ad.KB1M;
        s.npair = dim / 2;
        s.csplit = ars_csplit(s.npair, s.rblocks);
        s.c = nfk_make_const(K, -tail_bound, tail_bound, -tail_bound, tail_bound, 1, 1e-3, 1e-3, 1e-3);
        hipStream_t st = (hipStream_t)stream;
#define NFK_ARS_LAUNCH(h, t, k) \
    if (ad.d.KBH == h && ad.d.T1 == t && K == k) \
        return launch_ars<h, t, k>(s, ad, logdet, logdet_mode, (float)M_PI, (float)tail_bound, st);
        NFK_ARS_SHAPES(NFK_ARS_LAUNCH)
#undef NFK_ARS_LAUNCH
        return nfk_set_error("nfk_fused_ar: no kernel instance");
    }
    const ArDims d = ar_dims(hidden, K, dim);
    ArArgs a;
    a.x = x;
    a.pack = pack;
    a.out = out;
    a.logdet = logdet;
    a.status = status;
    a.ldx = ldx;
    a.ldo = ldo;
    a.batch = batch;
    a.dim = dim;
    a.mode = logdet_mode;
    a.sb = d.SB;
    a.kb1m = d.KB1M;
    a.nsr = ar_nsub(d, dim);
    a.pi = (float)M_PI;  // torch.tensor(np.pi) times an fp32 tensor: an fp32 product
    a.bnd = (float)tail_bound;
    // unconstrained_RQS(..., tail_bound=B) with the default minimum bin sizes (flows.py:186-187)
    a.c = nfk_make_const(K, -tail_bound, tail_bound, -tail_bound, tail_bound, 1, 1e-3, 1e-3, 1e-3);
    const bool inv = inverse != 0;
    // the column split needs the per-column log|det| workspace; without one
    // (or a smaller one) the launch keeps one range per workgroup
    a.csplit = ar_csplit(d, dim, batch, inv);
    if (a.csplit > 1 && (workspace == nullptr || workspace_floats < (int64_t)dim * batch)) a.csplit = 1;
    a.ld_cols = a.csplit > 1 ? workspace : nullptr;
    const int64_t per = (int64_t)ar_waves(d) * 16;
    a.rblocks = (batch + per - 1) / per;
    hipStream_t st = (hipStream_t)stream;
    int kbx = 0;
    ar_instance(d, K, &kbx);
#define NFK_AR_LAUNCH(h, t, k, xx) \
    if (d.KBH == h && d.T1 == t && K == k && kbx == xx) return launch_ar<h, t, k, xx>(a, d, inv, st);
    NFK_AR_SHAPES(NFK_AR_LAUNCH)
#undef NFK_AR_LAUNCH
    return nfk_set_error("nfk_fused_ar: no kernel instance");
}

// NSF_CL layers with a wide conditioner, reached through nfk_fused_nsf_* (nfk_fused.hip)
bool nfk_cl_ok(int n_lo, int n_up, int hidden, int K) { return cl_ok(n_lo, n_up, hidden, K); }

int64_t nfk_cl_pack_floats(int n_lo, int n_up, int hidden, int K) {
    return cl_ok(n_lo, n_up, hidden, K) ? cl_pack_floats(cl_dims(hidden, K, n_lo), n_up) : 0;
}

int nfk_cl_pack(const float* w0, const float* b0, const float* w2, const float* b2, const float* w4,
                const float* b4, int n_lo, int n_up, int hidden, int K, float* pack, hipStream_t st) {
    if (!cl_ok(n_lo, n_up, hidden, K)) return nfk_set_error("nfk_fused_nsf_pack: shape not supported");
    const ArDims d = cl_dims(hidden, K, n_lo);
    ClPackArgs a{w0, b0, w2, b2, w4, b4, pack, n_lo, n_up, hidden, K, (n_lo + 31) / 32, d};
    hipError_t e = hipMemsetAsync(pack, 0, 3 * sizeof(float), st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_cl_max, dim3(256), dim3(256), 0, st, a);
    int64_t g = (cl_pack_floats(d, n_up) + 255) / 256;
    if (g > 16384) g = 16384;
    hipLaunchKernelGGL(k_cl_pack, dim3((unsigned)g), dim3(256), 0, st, a);
    e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

int64_t nfk_cl_workspace(int n_lo, int n_up, int hidden, int K, int64_t batch) {
    if (!cl_ok(n_lo, n_up, hidden, K) || batch <= 0) return 0;
    return cl_csplit(n_up, batch) > 1 ? (int64_t)n_up * batch : 0;
}

int nfk_cl_launch(const float* x, int64_t ldx, const float* pack, const int32_t* up_in, const int32_t* up_out,
                  int n_up, const int32_t* lo_in, const int32_t* lo_out, int n_lo, int hidden, float* z, int64_t ldz,
                  float* logdet, int mode, int64_t batch, int K, double tail_bound, bool inv, int32_t* status,
                  float* workspace, int64_t workspace_floats, hipStream_t st) {
    if (!cl_ok(n_lo, n_up, hidden, K)) return nfk_set_error("nfk_fused_nsf: shape not supported");
    const ArDims d = cl_dims(hidden, K, n_lo);
    ClArgs a;
    a.x = x;
    a.pack = pack;
    a.z = z;
    a.logdet = logdet;
    a.status = status;
    a.up_in = up_in;
    a.up_out = up_out;
    a.lo_in = lo_in;
    a.lo_out = lo_out;
    a.ldx = ldx;
    a.ldz = ldz;
    a.batch = batch;
    a.n_lo = n_lo;
    a.n_up = n_up;
    a.mode = mode;
    a.sb = d.SB;
    a.kb1 = (n_lo + 31) / 32;
    a.csplit = cl_csplit(n_up, batch);
    if (a.csplit > 1 && (workspace == nullptr || workspace_floats < (int64_t)n_up * batch)) a.csplit = 1;
    a.ld_cols = a.csplit > 1 ? workspace : nullptr;
    a.rblocks = (batch + 63) / 64;
    // unconstrained_RQS(..., tail_bound=B) with the default minimum bin sizes (flows.py:236-237)
    a.c = nfk_make_const(K, -tail_bound, tail_bound, -tail_bound, tail_bound, 1, 1e-3, 1e-3, 1e-3);
#define NFK_CL_LAUNCH(h, t, k) \
    if (d.KBH == h && d.T1 == t && K == k) return launch_cl<h, t, k>(a, d, inv, st);
    NFK_CL_SHAPES(NFK_CL_LAUNCH)
#undef NFK_CL_LAUNCH
    return nfk_set_error("nfk_fused_nsf: no kernel instance");
}
