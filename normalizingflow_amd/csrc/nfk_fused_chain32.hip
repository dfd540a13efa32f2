// nfk_fused_chain32.hip -- the chained fused NSF_CL launch (nfk_fused_nsf_chain,
// nf/models.py:13-40 over nf/flows.py:227-253 layers) on 32x32x16 MFMAs.
//
// One wave owns 32 samples.  Every product is computed transposed on
// v_mfma_f32_32x32x16_f16, D[32 rows][32 samples] += A[32 rows][16 k] .
// B[16 k][32 samples], in the fp16 two-way split of the other fused kernels
// (hi + lo, three products, fp32 accumulation, power-of-two pre-scaling).
// Against the 16x16x32 chain (nfk_fused_chain2.hip) the matrix-pipe cycles
// per sample are the same, but there are half as many MFMA instructions (an
// MFMA holds the SIMD's vector issue for 8 cycles either way: 8 of 16 for
// 16x16x32, 8 of 32 for 32x32x16 -- MI355X_MICROARCH.md) and half the A
// fragments to read from LDS per flop.
// Operand maps (gfx950, lane l, s = l & 31, h = l >> 5): A[row s][k 8h + j],
// B[k 8h + j][col s], D register i = row 8 (i >> 2) + 4 h + (i & 3) of col s.
// So a layer's accumulator tile IS the next layer's B operand with no lane
// movement: registers 8u .. 8u + 7 form k-step u, element j of lane half h
// being row 16 u + 8 (j >> 2) + 4 h + (j & 3) -- the pack permutes the next
// layer's weight columns to that order.
//   hidden tiles (H = 97 .. 100): tiles 0..2 = features 32 T + row; tile 3
//     = the tail features 96 + (row & 3), every row duplicated, whose B
//     operand is one k-step holding {hi, lo} (lane half 0) and {hi, 0}
//     (half 1) of the four features against A = {lo, hi} / {hi, 0} of the
//     weights: all three split products in one MFMA;
//   output layer: per 8-coordinate chunk, the W, H and D logits as records of
//     two tiles (parameters 0..3, 4..7); row r of tile T = parameter
//     4 T + (r & 3) of coordinate 2 (r >> 3) + ((r >> 2) & 1), so lane (s, h)
//     holds all K parameters of coordinates 2 g + h, g = 0..3, of sample s
//     (registers 4 g .. 4 g + 3 of both tiles) and evaluates their splines
//     with the epilogue of the other fused kernels (knot_phase, epilogue C).
// Staging, barriers, maps, the x row tiles, the prior epilogue and the
// status words follow k_nsf_chain2; per layer 15 sub-records (layer 1
// whole, layer 2 in two halves, three records per 8-coordinate chunk).
// Results agree with the 16x16x32 kernels to fp32 rounding (the k sums run in
// another order), not bitwise.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "nfk_fused_impl.h"

namespace nfk_fused {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32(h8 a, h8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// pack geometry (c3 class: n_lo = 16 KS1, hidden 97..100, K <= 8, n_up % 8 == 0)
constexpr int k32KSF = 6;             // full k-steps of the hidden layers (96 features)
constexpr int k32SB = 27;             // blocks of a two-tile sub-record: 6 x 2 x 2 + 2 tail + bias
struct P32 {
    int KS1, NCH8, P, K, H, n_lo, n_up;
    int64_t o_l1, o_l2, o_l3, total;  // float offsets
};
__host__ __device__ inline P32 p32_layout(int n_lo, int n_up, int H, int K) {
    P32 p{};
    p.n_lo = n_lo;
    p.n_up = n_up;
    p.H = H;
    p.K = K;
    p.P = 3 * K - 1;
    p.KS1 = n_lo / 16;
    p.NCH8 = n_up / 8;
    p.o_l1 = 256;
    p.o_l2 = p.o_l1 + (int64_t)(8 * p.KS1 + 1) * 256;
    p.o_l3 = p.o_l2 + (int64_t)2 * k32SB * 256;
    p.total = p.o_l3 + (int64_t)p.NCH8 * 3 * k32SB * 256;
    return p;
}

bool chain32_shape_ok(int n_lo, int n_up, int H, int K) {
    return n_lo == 32 && n_up % 8 == 0 && n_up >= 8 && n_lo + n_up <= kMaxD && (n_lo + n_up) % 4 == 0 &&
           H >= 97 && H <= 100 && K == 8;
}

namespace {

// hidden feature of row r of hidden tile T (tile 3: the tail, duplicated)
__host__ __device__ inline int f32_hidden(int T, int r) { return T < 3 ? 32 * T + r : 96 + (r & 3); }
// contraction index of element j (lane half h) of full k-step ks over a hidden layer
__host__ __device__ inline int f32_kidx(int ks, int h, int j) {
    return 32 * (ks >> 1) + 16 * (ks & 1) + 8 * (j >> 2) + 4 * h + (j & 3);
}

struct Pack32Args {
    const float *w0, *b0, *w2, *b2, *w4, *b4;
    float* out;
    P32 p;
};

__global__ __launch_bounds__(256) void k_pack32_max(Pack32Args a) {
    const P32& p = a.p;
    const int64_t n1 = (int64_t)p.H * p.n_lo, n2 = (int64_t)p.H * p.H, n3 = (int64_t)p.n_up * p.P * p.H;
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
        unsigned int* hd = reinterpret_cast<unsigned int*>(a.out);
        atomicMax(hd, __float_as_uint(m1));
        atomicMax(hd + 1, __float_as_uint(m2));
        atomicMax(hd + 2, __float_as_uint(m3));
    }
}

__device__ int p32_scale_exp(float maxw) {
    if (!(maxw > 0.0f) || !(maxw < 3.0e38f)) return 0;
    int e;
    frexpf(maxw, &e);
    return 15 - e;
}

// word wl of block blk of a two-tile hidden-input sub-record (tiles T0, T0+1
// of an nt-tile record): [ks][tile][part] full k-steps, then [tile] tail
// blocks, then the bias block [tile][32 rows]
template <class ValF, class BiasF>
__device__ uint32_t p32_sub_word(int blk, int wl, int nt, int T0, float sc, float bsc, int H, ValF val, BiasF bias) {
    const int lane = wl >> 2, jp = 2 * (wl & 3), r = lane & 31, h = lane >> 5;
    if (blk < k32KSF * 4) {
        const int part = blk & 1, idx = blk >> 1, ks = idx >> 1, t = T0 + (idx & 1);
        if (t >= nt) return 0u;
        const int k0 = f32_kidx(ks, h, jp), k1 = f32_kidx(ks, h, jp + 1);
        return nfk_f16_part_pair(val(t, r, k0) * sc, val(t, r, k1) * sc, part);
    }
    if (blk < k32KSF * 4 + 2) {  // tail: h = 0 {lo, hi}, h = 1 {hi, 0} of features 96 .. 99
        const int t = T0 + (blk - k32KSF * 4);
        if (t >= nt) return 0u;
        float v[2];
        int part[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int j = jp + e;
            const int f = 96 + (j & 3);
            const float w = f < H ? val(t, r, f) * sc : 0.0f;
            if (h == 0) {
                v[e] = w;
                part[e] = j < 4 ? 1 : 0;
            } else {
                v[e] = j < 4 ? w : 0.0f;
                part[e] = 0;
            }
        }
        const _Float16 h0 = (_Float16)v[0], h1 = (_Float16)v[1];
        const _Float16 r0 = part[0] ? (_Float16)(v[0] - (float)h0) : h0;
        const _Float16 r1 = part[1] ? (_Float16)(v[1] - (float)h1) : h1;
        return (uint32_t)__builtin_bit_cast(uint16_t, r0) | ((uint32_t)__builtin_bit_cast(uint16_t, r1) << 16);
    }
    if (blk == k32KSF * 4 + 2) {
        const int t = T0 + (wl >> 5), rr = wl & 31;
        return __float_as_uint((wl >> 5) < 2 && t < nt ? bias(t, rr) * bsc : 0.0f);
    }
    return 0u;
}

__global__ __launch_bounds__(256) void k_pack32(Pack32Args a) {
    const P32& p = a.p;
    uint32_t* out = reinterpret_cast<uint32_t*>(a.out);
    const unsigned int* hd = reinterpret_cast<const unsigned int*>(a.out);
    const int s1 = p32_scale_exp(__uint_as_float(hd[0])), s2 = p32_scale_exp(__uint_as_float(hd[1])),
              s3 = p32_scale_exp(__uint_as_float(hd[2]));
    const float sc1 = ldexpf(1.0f, s1), sc2 = ldexpf(1.0f, s2), sc3 = ldexpf(1.0f, s3);
    const float bs2 = ldexpf(1.0f, s2 + 14), bs3 = ldexpf(1.0f, s3 + 14);
    const int H = p.H;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < p.total;
         g += (int64_t)gridDim.x * blockDim.x) {
        if (g < 256) {  // header: the 16x16 pack's (nfk_fused.hip pack_header)
            if (g == 3) out[g] = __float_as_uint(ldexpf(1.0f, -s1));
            else if (g == 4) out[g] = __float_as_uint(ldexpf(1.0f, -(s2 + 14)));
            else if (g == 5) out[g] = __float_as_uint(ldexpf(1.0f, -(s3 + 14)));
            else if (g >= 6) out[g] = 0u;
            continue;
        }
        uint32_t v = 0u;
        if (g < p.o_l2) {  // layer 1: [ks][tile (4)][part], bias [tile][32] unscaled
            const int64_t w = g - p.o_l1;
            const int blk = (int)(w >> 8), wl = (int)(w & 255);
            const int lane = wl >> 2, jp = 2 * (wl & 3), r = lane & 31, h = lane >> 5;
            if (blk < 8 * p.KS1) {
                const int part = blk & 1, idx = blk >> 1, ks = idx >> 2, t = idx & 3;
                const int f = f32_hidden(t, r);
                const int k0 = 16 * ks + 8 * h + jp;
                float v0 = 0.0f, v1 = 0.0f;
                if (f < H) {
                    v0 = a.w0[(int64_t)f * p.n_lo + k0] * sc1;
                    v1 = a.w0[(int64_t)f * p.n_lo + k0 + 1] * sc1;
                }
                v = nfk_f16_part_pair(v0, v1, part);
            } else {
                const int t = wl >> 5, rr = wl & 31;
                const int f = f32_hidden(t & 3, rr);
                v = __float_as_uint((t < 4 && f < H) ? a.b0[f] : 0.0f);
            }
        } else if (g < p.o_l3) {  // layer 2: two sub-records of two tiles
            const int64_t w = g - p.o_l2;
            const int sub = (int)(w / (k32SB * 256));
            const int blk = (int)((w >> 8) - (int64_t)sub * k32SB), wl = (int)(w & 255);
            v = p32_sub_word(
                blk, wl, 4, 2 * sub, sc2, bs2, H,
                [&](int t, int r, int k) -> float {
                    const int f = f32_hidden(t, r);
                    return (f < H && k < H) ? a.w2[(int64_t)f * H + k] : 0.0f;
                },
                [&](int t, int r) -> float {
                    const int f = f32_hidden(t, r);
                    return f < H ? a.b2[f] : 0.0f;
                });
        } else {  // output layer: per 8-coordinate chunk the W, H, D records
            const int64_t w = g - p.o_l3;
            const int rec = (int)(w / (k32SB * 256));
            const int blk = (int)((w >> 8) - (int64_t)rec * k32SB), wl = (int)(w & 255);
            const int c8 = rec / 3, ph = rec - 3 * c8;  // 0 W, 1 H, 2 D
            const int np = ph == 2 ? p.K - 1 : p.K, pbase = ph * p.K;
            auto rowpar = [&](int t, int r, int& jc, int& pr) {
                jc = 8 * c8 + 2 * (r >> 3) + ((r >> 2) & 1);
                pr = 4 * t + (r & 3);
            };
            v = p32_sub_word(
                blk, wl, 2, 0, sc3, bs3, H,
                [&](int t, int r, int k) -> float {
                    int jc, pr;
                    rowpar(t, r, jc, pr);
                    return (jc < p.n_up && pr < np && k < H) ? a.w4[((int64_t)jc * p.P + pbase + pr) * H + k] : 0.0f;
                },
                [&](int t, int r) -> float {
                    int jc, pr;
                    rowpar(t, r, jc, pr);
                    return (jc < p.n_up && pr < np) ? a.b4[(int64_t)jc * p.P + pbase + pr] : 0.0f;
                });
        }
        out[g] = v;
    }
}

// tanh (x 2^14, the split scale) of a hidden tile's accumulators into the
// next layer's B operands: full tiles T < 3 give k-steps 2 T, 2 T + 1; tile 3
// the tail operand
__device__ __forceinline__ void act32(f32x16 (&hd)[4], float c2, h8 (&bh)[k32KSF], h8 (&bl)[k32KSF], h8& btail,
                                      int h) {
#pragma unroll
    for (int T = 0; T < 3; ++T)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = tanh_scaled(hd[T][8 * u + j], c2);
                const _Float16 hh = (_Float16)v;
                bh[2 * T + u][j] = hh;
                bl[2 * T + u][j] = (_Float16)(v - (float)hh);
            }
    _Float16 th[4], tl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float v = tanh_scaled(hd[3][j], c2);
        th[j] = (_Float16)v;
        tl[j] = (_Float16)(v - (float)th[j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        btail[j] = th[j];
        btail[4 + j] = h == 0 ? tl[j] : (_Float16)0.0f;
    }
}

// one two-tile sub-record over a hidden input: acc[t] = bias + A_t . B
template <bool RING>
__device__ __forceinline__ void gemm32(const h8 (&bh)[k32KSF], const h8 (&bl)[k32KSF], h8 btail, const float4* slot,
                                       int lane, int h, f32x16 (&acc)[2]) {
    const float4* bias = slot + (k32KSF * 4 + 2) * 64;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {  // rows 8 g + 4 h + 0..3
            const float4 v = bias[t * 8 + 2 * g + h];
            acc[t][4 * g] = v.x;
            acc[t][4 * g + 1] = v.y;
            acc[t][4 * g + 2] = v.z;
            acc[t][4 * g + 3] = v.w;
        }
    float4 ring[RING ? 2 : 1][4];
    auto fetch = [&](int ks, float4 (&r)[4]) {
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = slot[(ks * 4 + j) * 64 + lane];
    };
    if (RING) fetch(0, ring[0]);
#pragma unroll
    for (int ks = 0; ks < k32KSF; ++ks) {
        if (RING) {  // A fragments of k-step ks + 1 in flight during ks
            if (ks + 1 < k32KSF) fetch(ks + 1, ring[(ks + 1) & (RING ? 1 : 0)]);
            __builtin_amdgcn_sched_barrier(0);
        } else {
            fetch(ks, ring[0]);
        }
        const float4* r = ring[ks & (RING ? 1 : 0)];
        const h8 ahi0 = __builtin_bit_cast(h8, r[0]), alo0 = __builtin_bit_cast(h8, r[1]);
        const h8 ahi1 = __builtin_bit_cast(h8, r[2]), alo1 = __builtin_bit_cast(h8, r[3]);
        acc[0] = mfma32(alo0, bh[ks], acc[0]);
        acc[1] = mfma32(alo1, bh[ks], acc[1]);
        acc[0] = mfma32(ahi0, bl[ks], acc[0]);
        acc[1] = mfma32(ahi1, bl[ks], acc[1]);
        acc[0] = mfma32(ahi0, bh[ks], acc[0]);
        acc[1] = mfma32(ahi1, bh[ks], acc[1]);
    }
    const h8 at0 = __builtin_bit_cast(h8, slot[(k32KSF * 4) * 64 + lane]);
    const h8 at1 = __builtin_bit_cast(h8, slot[(k32KSF * 4 + 1) * 64 + lane]);
    acc[0] = mfma32(at0, btail, acc[0]);
    acc[1] = mfma32(at1, btail, acc[1]);
}

}  // namespace

// NW waves per workgroup: 4 (two workgroups per CU, one slot), 8 (one
// workgroup, two slots) or 12 (one workgroup, three waves per SIMD, one slot)
constexpr int c32_slots(int nw) { return nw == 8 ? 2 : 1; }
inline size_t lds_bytes_chain32(int D, int K, int nl, int nw) {
    return (size_t)c32_slots(nw) * k32SB * 1024 + (size_t)((4 * nl + (nl + 1) * D + 15) / 16) * 16 +
           (size_t)nw * 32 * (D + 1) * sizeof(float) + (size_t)nw * K * 64 * sizeof(int);
}

namespace {

template <int K, bool INV, int NW>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void k_nsf_chain32(FusedArgs a) {
    constexpr bool RING = NW != 12;  // 12 waves: no A-fragment prefetch (168 VGPRs)
    constexpr int NSLOT = c32_slots(NW);
    constexpr bool DB = NSLOT == 2;  // double-buffered records, one barrier per record
    using ArgsK = const __attribute__((address_space(4))) FusedArgs;
    ArgsK* A = (ArgsK*)__builtin_amdgcn_kernarg_segment_ptr();
    (void)a;
    constexpr int KS1 = 2;  // n_lo = 32
    constexpr int DN = K - 1;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int s = lane & 31, h = lane >> 5;
    const int D = A->n_lo + A->n_up;
    extern __shared__ __attribute__((aligned(16))) float4 lds4[];
    float4* const slotA = lds4;
    float4* const slotB = lds4 + (NSLOT - 1) * k32SB * 64;
    const int NL = A->nlayers;
    int32_t* const cst = reinterpret_cast<int32_t*>(lds4 + NSLOT * k32SB * 64);
    uint8_t* const cm = reinterpret_cast<uint8_t*>(cst + NL);
    const uint8_t* c_lo = cm;
    const uint8_t* c_up = cm;
    const uint8_t* const c_src = cm + NL * D;
    const int XS = D + 1;
    float* const xbase = reinterpret_cast<float*>(lds4 + NSLOT * k32SB * 64 + (4 * NL + (NL + 1) * D + 15) / 16);
    float* const xt = xbase + wid * 32 * XS;  // this wave's 32 rows
    int* const scr = reinterpret_cast<int*>(xbase + NW * 32 * XS) + wid * K * 64;
    const int32_t pbase = A->o_h1;  // the pack32 follows the layer's 16x16 pack
    const float* pk = A->packs[0] + pbase;
    const int64_t b0 = ((int64_t)blockIdx.x * NW + wid) * 32;
    const int64_t rem = A->batch - b0;
    const int nall = rem <= 0 ? 0 : (rem < 32 ? (int)rem : 32);
    const bool row_ok = s < nall;
    const int NCH8 = A->n_up / 8;
    const int o_l2 = A->o_h2, o_l3 = A->o_w3;  // the pack32 offsets (floats)
    h8 bh[k32KSF], bl[k32KSF], btail;

    // sub-record sequence of a layer: 0 = layer 1 (8 KS1 + 1 blocks), 1-2 = layer 2
    // halves, then per chunk the searched, other and derivative records
    const int NSR = 3 + 3 * NCH8;
    int gsr = 0;              // records consumed (slot gsr & 1 in the two-slot form)
    int st_l = 0, st_q = 0;   // the next record to copy: layer, record of the layer
    int st_g = 0;             // ... and its index over the chain
    const float4* slot = slotA;  // the record the current GEMM reads
    auto stage_next = [&]() {
        if (st_l >= NL) return;
        const float* p = A->packs[st_l] + pbase;
        float4* dst = (st_g & 1) ? slotB : slotA;
        const int q = st_q;
        if (q == 0) {
            stage_record<NW>(p + 256, 8 * KS1 + 1, dst, wid, lane);
        } else if (q <= 2) {
            stage_record<NW>(p + o_l2 + (int64_t)(q - 1) * k32SB * 256, k32SB, dst, wid, lane);
        } else {
            const int u = q - 3, c8 = u / 3, v = u - 3 * c8;
            const int ph = v == 0 ? (INV ? 1 : 0) : (v == 1 ? (INV ? 0 : 1) : 2);
            stage_record<NW>(p + o_l3 + (int64_t)(3 * c8 + ph) * k32SB * 256, k32SB, dst, wid, lane);
        }
        ++st_g;
        if (++st_q == NSR) {
            st_q = 0;
            ++st_l;
        }
    };
    // One slot: a GEMM step ends at a barrier after which the next record's
    // copy is issued; the epilogue step after it ends at the barrier that waits
    // for it.  Two slots: the copy of record g + 2 is issued after the barrier
    // ending GEMM g (slot g & 1 free) and waited for before the barrier ending
    // GEMM g + 1, so that barrier is the only one per record.
    auto gemm_end = [&](bool last) {
        if (DB)
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        else
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
#ifndef NFK_ABL_NOSTAGE  // diagnostic: no record copies after the prologue
        stage_next();
#endif
        ++gsr;
        slot = (DB && (gsr & 1)) ? slotB : slotA;
        if (!DB && !last) {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
    };
    auto epi_end = [&]() {
        if (DB) return;
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };

    // ---- prologue
    float ld_acc = (h == 0 && row_ok && A->mode == 2) ? A->logdet[b0 + s] : 0.0f;
    if (nall > 0) {
        const uint32_t base = lds_addr(xt);
        for (int r = 0; r < 32; ++r) {
            const float* src = A->x + (b0 + (r < nall ? r : 0)) * A->ldx;
            for (int c0 = 0; c0 < D; c0 += 64)
                if (c0 + lane < D) dma4(src + c0 + lane, base + (r * XS + c0) * 4);
        }
    }
    stage_next();
    if (DB) stage_next();
    for (int i = threadIdx.x; i < (NL + 1) * D; i += 64 * NW) cm[i] = (uint8_t)A->cmaps[i];
    if ((int)threadIdx.x < NL) cst[threadIdx.x] = 0;
    dma_barrier();

    for (int l = 0; l < NL; ++l) {
        asm volatile("" : "+s"(A));
        pk = A->packs[l] + pbase;
        c_lo = cm + l * D;
        c_up = c_lo + A->n_lo;
        const FusedConst c = *(const FusedConst*)&A->c;  // by value: SGPRs for the layer
        const float un1 = pk[3], un2 = pk[4], un3 = pk[5];
        bool any_in = false, any_nd = false;

        // ---- layer 1: B = x at the lower coordinates 16 ks + 8 h + j of sample s
        {
            f32x16 h1[4];
            float e[KS1][8];
            float mx = 0.0f;
            const float* xr = xt + s * XS;
#pragma unroll
            for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    e[ks][j] = xr[c_lo[16 * ks + 8 * h + j]];
                    mx = fmaxf(mx, fabsf(e[ks][j]));
                }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
            int ex = 0;
            if (mx > 0.0f && mx < 3.0e38f) frexpf(mx, &ex);
            const float sx = ldexpf(1.0f, 14 - ex);
            const float unx = ldexpf(un1, ex - 14);
            const float bsc = sx / un1;
            const float4* bias = slot + 8 * KS1 * 64;
#pragma unroll
            for (int T = 0; T < 4; ++T)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const float4 v = bias[T * 8 + 2 * g + h];
                    h1[T][4 * g] = v.x * bsc;
                    h1[T][4 * g + 1] = v.y * bsc;
                    h1[T][4 * g + 2] = v.z * bsc;
                    h1[T][4 * g + 3] = v.w * bsc;
                }
            h8 xh[KS1], xl[KS1];
#pragma unroll
            for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float v = e[ks][j] * sx;
                    const _Float16 hh = (_Float16)v;
                    xh[ks][j] = hh;
                    xl[ks][j] = (_Float16)(v - (float)hh);
                }
#pragma unroll
            for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
                for (int T = 0; T < 4; ++T) {
                    const h8 ahi = __builtin_bit_cast(h8, slot[((ks * 4 + T) * 2) * 64 + lane]);
                    const h8 alo = __builtin_bit_cast(h8, slot[((ks * 4 + T) * 2 + 1) * 64 + lane]);
                    h1[T] = mfma32(alo, xh[ks], h1[T]);
                    h1[T] = mfma32(ahi, xl[ks], h1[T]);
                    h1[T] = mfma32(ahi, xh[ks], h1[T]);
                }
            gemm_end(true);
            act32(h1, -2.0f * kL2E * unx, bh, bl, btail, h);
        }
        epi_end();
        // ---- layer 2: two sub-records of two tiles
        {
            f32x16 h2[4];
            {
                f32x16 acc[2];
                gemm32<RING>(bh, bl, btail, slot, lane, h, acc);
                h2[0] = acc[0];
                h2[1] = acc[1];
            }
            gemm_end(false);
            {
                f32x16 acc[2];
                gemm32<RING>(bh, bl, btail, slot, lane, h, acc);
                h2[2] = acc[0];
                h2[3] = acc[1];
            }
            gemm_end(true);
            act32(h2, -2.0f * kL2E * un2, bh, bl, btail, h);
        }
        epi_end();

        const float l2e3 = kL2E * un3;
        float ldsum = 0.0f;
        int jj4[4];
        float xv[4];
        int kb[4];
        float cw_k[4], w_k[4], ch_k[4], h_k[4];
        for (int c8 = 0; c8 < NCH8; ++c8) {
            // lane (s, h): coordinates 8 c8 + 2 g + h, g = 0..3
#pragma unroll
            for (int g = 0; g < 4; ++g) jj4[g] = 8 * c8 + 2 * g + h;
            {
                f32x16 acc[2];
                gemm32<RING>(bh, bl, btail, slot, lane, h, acc);
                gemm_end(true);
                f32x4 u4[K];
#pragma unroll
                for (int p = 0; p < K; ++p)
#pragma unroll
                    for (int g = 0; g < 4; ++g) u4[p][g] = p < 4 ? acc[0][4 * g + p] : acc[1][4 * g + p - 4];
#pragma unroll
                for (int g = 0; g < 4; ++g) xv[g] = xt[s * XS + c_up[jj4[g]]];
                knot_phase<K, true, 0, 4, true>(u4, xv, c, l2e3, kb, INV ? ch_k : cw_k, INV ? h_k : w_k, scr, lane);
            }
            epi_end();
            {
                f32x16 acc[2];
                gemm32<RING>(bh, bl, btail, slot, lane, h, acc);
                gemm_end(true);
                f32x4 u4[K];
#pragma unroll
                for (int p = 0; p < K; ++p)
#pragma unroll
                    for (int g = 0; g < 4; ++g) u4[p][g] = p < 4 ? acc[0][4 * g + p] : acc[1][4 * g + p - 4];
                knot_phase<K, false, 0, 4, true>(u4, xv, c, l2e3, kb, INV ? cw_k : ch_k, INV ? w_k : h_k, scr, lane);
            }
            epi_end();
            {
                f32x16 acc[2];
                gemm32<RING>(bh, bl, btail, slot, lane, h, acc);
                gemm_end(true);
                float* fs = reinterpret_cast<float*>(scr);
#ifdef NFK_ABL_NOEPI  // diagnostic: the spline replaced by a sum
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    float v = cw_k[g] + w_k[g] + ch_k[g] + h_k[g];
#pragma unroll
                    for (int j = 0; j < 8; ++j) v += acc[j >> 2][4 * g + (j & 3)];
                    xt[s * XS + c_up[jj4[g]]] = v;
                    ldsum += v;
                    any_in = true;
                }
                if (false)
#endif
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    // epilogue C of k_fused_nsf, op for op
                    const int k = kb[g];
#pragma unroll
                    for (int j = 0; j < DN; ++j) fs[j * 64 + lane] = j < 4 ? acc[0][4 * g + j] : acc[1][4 * g + j - 4];
                    const float raw_k = fs[(k > 0 ? k - 1 : 0) * 64 + lane];
                    const float raw_k1 = fs[(k < K - 1 ? k : K - 2) * 64 + lane];
                    const float dv_k = nfk_deriv_lean(raw_k * un3, c.min_d);
                    const float dv_k1 = nfk_deriv_lean(raw_k1 * un3, c.min_d);
                    const float d_k = (k == 0) ? c.d_edge : dv_k;
                    const float d_k1 = (k == K - 1) ? c.d_edge : dv_k1;
                    const float x = xv[g];
                    const float rw = nfk_rcp_fast(w_k[g]);
                    const float delta = h_k[g] * rw;
                    const float gap = (d_k + d_k1) - 2.0f * delta;
                    float out, th;
                    bool nd = false;
                    if (INV) {
                        const float y = x - ch_k[g];
                        const float qa = y * gap + h_k[g] * (delta - d_k);
                        const float qb = h_k[g] * d_k - y * gap;
                        const float qc = (-delta) * y;
                        const float disc = qb * qb - (4.0f * qa) * qc;
                        nd = !(disc >= 0.0f);
                        const float root = nfk_div<true>(2.0f * qc, -qb - sqrtf(disc));
                        out = root * w_k[g] + cw_k[g];
                        th = root;
                    } else {
                        th = (x - cw_k[g]) * rw;
                    }
                    const float t1mt = th * (1.0f - th);
                    const float den = delta + gap * t1mt;
                    if (!INV) {
                        const float num = h_k[g] * (delta * (th * th) + d_k * t1mt);
                        out = ch_k[g] + nfk_div<true>(num, den);
                    }
                    const float omt = 1.0f - th;
                    const float dnum =
                        (delta * delta) * ((d_k1 * (th * th) + (2.0f * delta) * t1mt) + d_k * (omt * omt));
                    float lad = (__builtin_amdgcn_logf(dnum) - 2.0f * __builtin_amdgcn_logf(den)) * kLN2;
                    lad = INV ? -lad : lad;
                    const bool inside = (x >= c.lo) && (x <= c.hi);
                    const bool live = jj4[g] < A->n_up && row_ok;
                    out = inside ? out : x;
                    xt[s * XS + c_up[jj4[g]]] = out;
                    ldsum += (inside && live) ? lad : 0.0f;
                    any_in |= inside && live;
                    any_nd |= nd && inside && live;
                }
            }
            epi_end();
        }
        // end of the layer: this sample's log|det| (both lane halves), status bits
        ld_acc = ld_acc + (ldsum + __shfl_xor(ldsum, 32, 64));
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
    if (h == 0 && row_ok && A->mode != 0) A->logdet[b0 + s] = ld_acc;
    if (A->log_prob != nullptr) {
        const float* row = xt + s * XS;
        const float il = A->prior_inv_scale;
        float m = 0.0f;
        for (int g4 = h; g4 < D4; g4 += 2) {
            const int o = 4 * g4;
            const float y0 = row[c_src[o]] * il, y1 = row[c_src[o + 1]] * il;
            const float y2 = row[c_src[o + 2]] * il, y3 = row[c_src[o + 3]] * il;
            m += (y0 * y0 + y1 * y1) + (y2 * y2 + y3 * y3);
        }
        m += __shfl_xor(m, 32, 64);
        const float lp = -0.5f * (A->prior_c2pi + m) - A->prior_hld;
        if (h == 0 && row_ok) A->log_prob[b0 + s] = lp + ld_acc;
        if (__any(row_ok && m != m) && lane == 0) atomicOr(cst, NFK_ST_NAN_Z);
    }
    __syncthreads();
    if (A->status != nullptr && (int)threadIdx.x < NL) {
        const int bits = cst[threadIdx.x];
        if (bits != 0 && (A->status[threadIdx.x] & bits) != bits) atomicOr(A->status + threadIdx.x, bits);
    }
}

}  // namespace

// waves per workgroup: NFK_C32_WAVES=12 in the environment selects the
// one-workgroup-per-CU form
static int chain32_waves() {
    static const int nw = [] {
        const char* e = std::getenv("NFK_C32_WAVES");
        if (e != nullptr && e[0] == '1' && e[1] == '2') return 12;
        return (e != nullptr && e[0] == '8') ? 8 : 4;
    }();
    return nw;
}

int64_t chain32_pack_floats(int n_lo, int n_up, int H, int K) {
    if (!chain32_shape_ok(n_lo, n_up, H, K)) return 0;
    return p32_layout(n_lo, n_up, H, K).total;
}

int chain32_pack(const float* w0, const float* b0, const float* w2, const float* b2, const float* w4,
                 const float* b4, int n_lo, int n_up, int H, int K, float* pack, hipStream_t st) {
    Pack32Args a{w0, b0, w2, b2, w4, b4, pack, p32_layout(n_lo, n_up, H, K)};
    hipError_t e = hipMemsetAsync(pack, 0, 3 * sizeof(float), st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_pack32_max, dim3(64), dim3(256), 0, st, a);
    int64_t g = (a.p.total + 255) / 256;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_pack32, dim3((unsigned)g), dim3(256), 0, st, a);
    e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

// a: the chain's FusedArgs; each layer's pack32 starts base floats into its
// pack (o_h1), o_h2 / o_w3 carry the pack32 layer-2 / output-layer offsets
int launch_chain32(FusedArgs a, int K, bool inv, int64_t base, hipStream_t st) {
    const P32 p = p32_layout(a.n_lo, a.n_up, 100, K);
    a.o_h1 = (int32_t)base;
    a.o_h2 = (int32_t)p.o_l2;
    a.o_w3 = (int32_t)p.o_l3;
    a.slot_blocks = k32SB;
    const int nw = chain32_waves();
    const int64_t per = (int64_t)nw * 32;
    const int64_t blocks = (a.batch + per - 1) / per;
    if (blocks == 0) return 0;
    const size_t lds = lds_bytes_chain32(a.n_lo + a.n_up, K, a.nlayers, nw);
    const dim3 g((unsigned)blocks), b(64 * nw);
    if (K != 8) return -1;
    if (nw == 12) {
        if (inv)
            hipLaunchKernelGGL((k_nsf_chain32<8, true, 12>), g, b, lds, st, a);
        else
            hipLaunchKernelGGL((k_nsf_chain32<8, false, 12>), g, b, lds, st, a);
    } else if (nw == 8) {
        if (inv)
            hipLaunchKernelGGL((k_nsf_chain32<8, true, 8>), g, b, lds, st, a);
        else
            hipLaunchKernelGGL((k_nsf_chain32<8, false, 8>), g, b, lds, st, a);
    } else {
        if (inv)
            hipLaunchKernelGGL((k_nsf_chain32<8, true, 4>), g, b, lds, st, a);
        else
            hipLaunchKernelGGL((k_nsf_chain32<8, false, 4>), g, b, lds, st, a);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

bool chain32_ok(int n_lo, int n_up, int H, int K, int nl) {
    const int nw = chain32_waves();
    return chain32_shape_ok(n_lo, n_up, H, K) &&
           (nw == 4 ? 2 : 1) * lds_alloc(lds_bytes_chain32(n_lo + n_up, K, nl, nw)) <= (size_t)kLdsBytes;
}

}  // namespace nfk_fused
