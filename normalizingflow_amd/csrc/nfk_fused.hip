// nfk_fused.hip -- one launch per NSF coupling layer: conditioner MLP
// (FCNN, nf/flows.py:20-35) on MFMA + rational-quadratic spline epilogue
// (nf/flows.py:227-253, nf/utils.py:27-152).  The [B, n_up, 3K-1] conditioner
// output never leaves registers.
//
// Work decomposition: one wave owns a tile of 16 samples.  All products are
// computed transposed, h^T[feature][sample] = W . act^T:
//   A operand = weights (from an LDS slot), B operand = activations (registers),
//   D: lane l, register r = output row 4*(l>>4)+r of sample l&15.
// Every layer runs as a two-way fp16 split on v_mfma_f32_16x16x32_f16 (layer
// 1 too, since round 4: x, of any magnitude, is first scaled per SAMPLE by a
// power of two 2^(14 - e), e from the max |x| over that sample's lower
// coordinates, clamped at e >= -64, the accumulators unscaled by the same
// factor): v = hi + lo with hi = f16(v), lo = f16(v - hi)
// (22 significant bits), product = lo.hi + hi.lo + hi.hi accumulated in fp32,
// dropping lo.lo (2^-22 relative).  Weights are pre-scaled by a power of two
// so that max|W| lies in [2^14, 2^15) and activations (tanh outputs) by 2^14,
// which keeps both parts in fp16's normal range; the exact power-of-two scale
// is undone inside the consumers (tanh constant, softmax log2e, softplus
// argument).  Accuracy matches the fp32 chain (mean |err| ~1e-7 on the
// logits); the fp16 form needs 3 x 16 MFMA cycles per 16x16x32 block where
// fp32 needs 8 x 32 -- and on gfx950 fp32 MFMA and VALU share one issue port
// (tools/ubench_coexec.hip), so MFMA cycles are paid in full.
//
// Hidden features are permuted (hid_feature in nfk_fused_impl.h) so that the
// accumulators of one layer ARE the B fragments of the next: no LDS round trip.
// Output layer: per chunk of 16 coordinates the 3K-1 parameter tiles are
// produced in three phases (W logits, H logits, D logits; H first when
// inverting).  Row i of a parameter tile is coordinate jbase + i, so lane l
// holds, for sample l&15, all K logits of coordinates jbase + 4q + r in
// registers and evaluates the spline there (nfk_spline.h lean forms).
// Per-sample log|det| is reduced across the four lane groups with xor-16/32
// shuffles.  Weights stream through two LDS slots (global_load_lds, one
// barrier per phase); each record is read from L2 once per 128 samples.
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
#include "nfk_fused_wide.h"

using namespace nfk_fused;

namespace nfk_fused {
#define NFK_X(h, t) NFK_FUSED_K(NFK_FUSED_EXTERN, h, t)
NFK_FUSED_KB(NFK_X)
#undef NFK_X
#define NFK_X(h) NFK_WIDE_K(NFK_WIDE_EXTERN, h)
NFK_WIDE_KB(NFK_X)
#undef NFK_X
}  // namespace nfk_fused

namespace {

struct PackArgs {
    const float *w0, *b0, *w2, *b2, *w4, *b4;
    float* out;
    Layout L;
};

// max |W| of layers 1, 2, 3 into hdr[0..2] as uint bits (non-negative floats
// order like their bit patterns)
__global__ __launch_bounds__(256) void k_pack_max(PackArgs a) {
    const Layout& L = a.L;
    const int64_t n1 = (int64_t)L.H * L.n_lo, n2 = (int64_t)L.H * L.H, n3 = (int64_t)L.n_up * L.P * L.H;
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

// power-of-two exponent s with max|W| 2^s in [2^14, 2^15)
__device__ int scale_exp(float maxw) {
    if (!(maxw > 0.0f) || !(maxw < 3.0e38f)) return 0;
    int e;
    frexpf(maxw, &e);  // maxw = m 2^e, m in [0.5, 1)
    return 15 - e;
}

__device__ uint32_t f16_part_pair(float v0, float v1, int part) {
    const _Float16 h0 = (_Float16)v0, h1 = (_Float16)v1;
    const _Float16 r0 = part ? (_Float16)(v0 - (float)h0) : h0;
    const _Float16 r1 = part ? (_Float16)(v1 - (float)h1) : h1;
    return (uint32_t)__builtin_bit_cast(uint16_t, r0) | ((uint32_t)__builtin_bit_cast(uint16_t, r1) << 16);
}

// word of an f16-split record (f16 blocks, tail blocks, bias block) with
// nt tiles; row(t, i) and the weight row pointer come from the caller's lambda
template <class RowF, class BiasF>
__device__ uint32_t pack_record_word(int blk, int wl, const Layout& L, int nt, float sc, float bsc,
                                     RowF row_of, BiasF bias_of) {
    const int nf = L.KBH * nt * 2, ntg = L.T1 ? (nt + 1) / 2 : 0;
    if (blk < nf) {
        const int part = blk & 1, idx = blk >> 1, kb = idx / nt, t = idx - kb * nt;
        const int lane = wl >> 2, j = 2 * (wl & 3);
        const int k0 = 32 * kb + 8 * (lane >> 4) + j;
        const float* w = row_of(t, lane & 15);
        float v0 = 0.0f, v1 = 0.0f;
        if (w != nullptr) {
            const int klim = L.T1 ? 32 * L.KBH : L.H;  // the tail step owns k >= 32 KBH
            if (k0 < klim && k0 < L.H) v0 = w[k0] * sc;
            if (k0 + 1 < klim && k0 + 1 < L.H) v1 = w[k0 + 1] * sc;
        }
        return f16_part_pair(v0, v1, part);
    }
    if (blk < nf + ntg) return tail_word(blk - nf, wl, nt, 32 * L.KBH, L.H, sc, row_of);
    const int t = wl >> 4, i = wl & 15;  // bias block [tile][row]
    return __float_as_uint(t < nt ? bias_of(t, i) * bsc : 0.0f);
}

struct PackScales {
    float sc1, sc2, sc3, bs2, bs3;
};

// Word g (>= L.o_h1) of the record layout (nfk_fused_impl.h).
__device__ uint32_t pack_word(const PackArgs& a, int64_t g, const PackScales& ps) {
    const Layout& L = a.L;
    const float sc1 = ps.sc1, sc2 = ps.sc2, sc3 = ps.sc3, bs2 = ps.bs2, bs3 = ps.bs3;
    const int kbh = L.KBH;
    if (g < L.o_h2) {  // layer 1: KB1 f16 k-blocks over the n_lo inputs + unscaled bias
        const int64_t w = g - L.o_h1;
        const int blk = (int)(w >> 8), wl = (int)(w & 255);
        if (blk < L.KB1 * L.HT * 2) {
            const int part = blk & 1, idx = blk >> 1, kb = idx / L.HT, t = idx - kb * L.HT;
            const int lane = wl >> 2, j = 2 * (wl & 3);
            const int f = hid_feature(t, lane & 15, kbh), k0 = 32 * kb + 8 * (lane >> 4) + j;
            float v0 = 0.0f, v1 = 0.0f;
            if (f < L.H) {
                if (k0 < L.n_lo) v0 = a.w0[(int64_t)f * L.n_lo + k0] * sc1;
                if (k0 + 1 < L.n_lo) v1 = a.w0[(int64_t)f * L.n_lo + k0 + 1] * sc1;
            }
            return f16_part_pair(v0, v1, part);
        } else {
            const int t = wl >> 4, f = hid_feature(t, wl & 15, kbh);
            return __float_as_uint((t < L.HT && f < L.H) ? a.b0[f] : 0.0f);
        }
    }
    if (g < L.o_w3) {  // layer 2
        const int64_t w = g - L.o_h2;
        return pack_record_word(
            (int)(w >> 8), (int)(w & 255), L, L.HT, sc2, bs2,
            [&](int t, int i) -> const float* {
                const int f = hid_feature(t, i, kbh);
                return f < L.H ? a.w2 + (int64_t)f * L.H : nullptr;
            },
            [&](int t, int i) -> float {
                const int f = hid_feature(t, i, kbh);
                return f < L.H ? a.b2[f] : 0.0f;
            });
    }
    // output layer: chunk, phase (W, H, D)
    const int64_t w3 = g - L.o_w3;
    const int64_t bl = w3 >> 8;
    const int chunk = (int)(bl / L.blk_chunk);
    int b = (int)(bl - (int64_t)chunk * L.blk_chunk);
    int nt = L.wide ? (L.K + 1) / 2 : L.K, pbase = 0, np = L.K;
    if (b >= L.blk_w) {
        b -= L.blk_w;
        pbase = L.K;
        if (b >= L.blk_w) {
            b -= L.blk_w;
            pbase = 2 * L.K;
            nt = L.wide ? L.K / 2 : L.K - 1;
            np = L.K - 1;
        }
    }
    // (coordinate, parameter) of row i of tile t (Layout: wide form or 16-coordinate form)
    auto coord = [&](int i) { return L.wide ? 8 * chunk + 2 * (i >> 2) + ((i >> 1) & 1) : 16 * chunk + i; };
    auto param = [&](int t, int i) { return L.wide ? 2 * t + (i & 1) : t; };
    return pack_record_word(
        b, (int)(w3 & 255), L, nt, sc3, bs3,
        [&](int t, int i) -> const float* {
            const int jc = coord(i), p = param(t, i);
            return (jc < L.n_up && p < np) ? a.w4 + ((int64_t)jc * L.P + pbase + p) * L.H : nullptr;
        },
        [&](int t, int i) -> float {
            const int jc = coord(i), p = param(t, i);
            return (jc < L.n_up && p < np) ? a.b4[(int64_t)jc * L.P + pbase + p] : 0.0f;
        });
}

// header words: the unscale factors (words 0-2 hold the maxima), and the scales
__device__ PackScales pack_header(const PackArgs& a, int64_t g) {
    const unsigned int* hdr = reinterpret_cast<const unsigned int*>(a.out);
    const int s1 = scale_exp(__uint_as_float(hdr[0])), s2 = scale_exp(__uint_as_float(hdr[1])),
              s3 = scale_exp(__uint_as_float(hdr[2]));
    uint32_t* out = reinterpret_cast<uint32_t*>(a.out);
    if (g == 3) out[g] = __float_as_uint(ldexpf(1.0f, -s1));
    if (g == 4) out[g] = __float_as_uint(ldexpf(1.0f, -(s2 + 14)));
    if (g == 5) out[g] = __float_as_uint(ldexpf(1.0f, -(s3 + 14)));
    if (g >= 6 && g < 256) out[g] = 0;
    return PackScales{ldexpf(1.0f, s1), ldexpf(1.0f, s2), ldexpf(1.0f, s3), ldexpf(1.0f, s2 + 14),
                      ldexpf(1.0f, s3 + 14)};
}

// One thread per packed 32-bit word (layout described in nfk_fused_impl.h).
__global__ __launch_bounds__(256) void k_pack(PackArgs a) {
    uint32_t* out = reinterpret_cast<uint32_t*>(a.out);
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < a.L.total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const PackScales ps = pack_header(a, g);
        if (g >= a.L.o_h1) out[g] = pack_word(a, g, ps);
    }
}

// Frame stream of the wide kernel (nfk_fused_wide.h): after the header, one
// 65-block frame per forward sub-step: the sub-record's blocks, zero padding,
// and at block 64 its record's bias block (every frame carries it; the kernel
// reads it only for the first sub-record of a record).  Words come from the
// record layout a.L (wide form) through pack_word.
__global__ __launch_bounds__(256) void k_pack_frames(PackArgs a, int s1, int ns, int gh, int gc) {
    const Layout& L = a.L;
    uint32_t* out = reinterpret_cast<uint32_t*>(a.out);
    const int64_t total = 256 + (int64_t)ns * kWideSlotBlocks * 256;
    const int s2 = L.KBH / gh, sc = L.KBH / gc;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const PackScales ps = pack_header(a, g);
        if (g < 256) continue;
        const int64_t w = g - 256;
        const int f = (int)(w / (kWideSlotBlocks * 256)), fw = (int)(w - (int64_t)f * kWideSlotBlocks * 256);
        const int blk = fw >> 8, wl = fw & 255;
        int64_t rec;
        int nt, j, nkb, gg;
        if (f < s1) {
            rec = L.o_h1, nt = L.HT, j = f, nkb = L.KB1, gg = gh;
        } else if (f < s1 + s2) {
            rec = L.o_h2, nt = L.HT, j = f - s1, nkb = L.KBH, gg = gh;
        } else {
            const int u = f - s1 - s2, ch = u / (3 * sc), v = u - ch * (3 * sc), part = v / sc;
            j = v - part * sc;
            rec = L.o_w3 + ((int64_t)ch * L.blk_chunk + part * L.blk_w) * 256;
            nt = L.K / 2, nkb = L.KBH, gg = gc;
        }
        const int kb0 = gg * j, nk = (nkb - kb0) < gg ? (nkb - kb0) : gg;
        uint32_t v = 0;
        if (blk == kWideFB)
            v = pack_word(a, rec + (int64_t)nkb * nt * 2 * 256 + wl, ps);
        else if (blk < nk * nt * 2)
            v = pack_word(a, rec + ((int64_t)kb0 * nt * 2 + blk) * 256 + wl, ps);
        out[g] = v;
    }
}

bool shape_ok(int n_lo, int n_up, int H, int K) {
    if (n_lo < 1 || n_up < 1 || n_lo + n_up > kMaxD || H < 1 || K < 2) return false;
    const Layout L = make_layout(n_lo, n_up, H, K);
    if (lds_bytes(L) > (size_t)kLdsBytes) return false;
    if (L.K > 16 || L.HT > 16) return false;  // one bias block per record
    bool kb = false, kk = false;
#define CHK_KB(h, t) kb |= (L.KBH == h && L.T1 == t);
    NFK_FUSED_KB(CHK_KB)
#undef CHK_KB
#define CHK_K(h, t, k) kk |= (K == k);
    NFK_FUSED_K(CHK_K, 0, 0)
#undef CHK_K
    return kb && kk;
}

// Shapes of the wide kernel (nfk_fused_wide.h): H = 32 KBH for an instantiated
// KBH, no tail step; layer-1 inputs within the KBH k-blocks; every lower
// coordinate inside the x tiles (16 lower + 16 upper coordinates per chunk
// pair); even K; LDS within the CU.
bool wide_ok(int n_lo, int n_up, int H, int K) {
    if (n_lo < 1 || n_up < 1 || H < 1 || K < 2 || (K & 1)) return false;
    const Layout L = make_layout(n_lo, n_up, H, K, 1);
    if (L.T1 != 0 || L.KB1 > L.KBH || n_lo > 16 * ((L.NCH + 1) / 2)) return false;
    if (kWideWGs * lds_alloc(wide_lds_bytes(n_lo, n_up)) > (size_t)kLdsBytes) return false;
    bool kb = false, kk = false;
#define CHK_KB(h) kb |= (L.KBH == h);
    NFK_WIDE_KB(CHK_KB)
#undef CHK_KB
#define CHK_K(h, k) kk |= (K == k);
    NFK_WIDE_K(CHK_K, 0)
#undef CHK_K
    return kb && kk;
}

// narrow kernel first (c3-class layers), the wide one for what it rejects
bool pack_ok(int n_lo, int n_up, int H, int K) { return shape_ok(n_lo, n_up, H, K) || wide_ok(n_lo, n_up, H, K); }

// the record layout of the kernel that will run this shape
Layout pack_layout(int n_lo, int n_up, int H, int K) {
    return make_layout(n_lo, n_up, H, K, shape_ok(n_lo, n_up, H, K) ? 0 : 1);
}

// floats of the pack: the record layout (narrow kernel) or header + frames (wide)
int64_t pack_floats(int n_lo, int n_up, int H, int K) {
    const Layout L = pack_layout(n_lo, n_up, H, K);
    if (!L.wide) return L.total;
    int s1;
    const int ns = wide_substeps(L.KB1, L.KBH, K, L.NCH, &s1);
    return 256 + (int64_t)ns * kWideSlotBlocks * 256;
}

uint32_t* g_trace = nullptr;  // diagnostic timeline buffer (NFK_TRACE builds)
int g_form = -1;            // nfk_debug_fused_form
int g_chain_form = -1;      // nfk_debug_chain_form
constexpr int kChainFormDefault = 1;  // nfk_fused_nsf_chain's kernel form
int g_last_chain_form = -1;           // nfk_debug_last_chain_form

int launch_wide(const FusedArgs& f, const Layout& L, int K, bool inv, hipStream_t st) {
    WideArgs a;
    a.trace = g_trace;
    a.x = f.x;
    a.pack = f.pack;
    a.up_in = f.up_in;
    a.up_out = f.up_out;
    a.lo_in = f.lo_in;
    a.lo_out = f.lo_out;
    a.z = f.z;
    a.logdet = f.logdet;
    a.status = f.status;
    a.ldx = f.ldx;
    a.ldz = f.ldz;
    a.batch = f.batch;
    a.n_lo = L.n_lo;
    a.n_up = L.n_up;
    a.KB1 = L.KB1;
    a.NCH = L.NCH;
    a.mode = f.mode;
    a.NS = wide_substeps(L.KB1, L.KBH, K, L.NCH, &a.S1);
    a.c = f.c;
    const size_t lds = wide_lds_bytes(L.n_lo, L.n_up);
#define DISPATCH(h, k) \
    if (L.KBH == h && K == k) return launch_fused_wide<h, k>(a, lds, inv, st);
#define DISPATCH_KB(h) NFK_WIDE_K(DISPATCH, h)
    NFK_WIDE_KB(DISPATCH_KB)
#undef DISPATCH_KB
#undef DISPATCH
    return nfk_set_error("nfk_fused_nsf: no wide kernel instance");
}

}  // namespace

// Diagnostic: timeline buffer for -DNFK_TRACE builds (not part of include/nfk.h).
extern "C" int nfk_debug_trace(void* buf) {
    g_trace = static_cast<uint32_t*>(buf);
    return 0;
}

// Diagnostic: form of k_fused_nsf: -1 = automatic (split where it fits unless
// NFK_FUSED_SPLIT=0), 0 = whole records, 1 = split where it fits.  Returns the
// previous setting.  Not part of include/nfk.h.
extern "C" int nfk_debug_fused_form(int form) {
    const int prev = g_form;
    g_form = form < 0 ? -1 : (form ? 1 : 0);
    return prev;
}

// Diagnostic: kernel of nfk_fused_nsf_chain: -1 = automatic (NFK_CHAIN_FORM in
// the environment, else the default of nfk_fused_nsf_chain), 0 = one
// 16-sample tile per wave, 1 = two tiles per wave (where instanced; else
// form 0).  Returns the previous setting.  Not part of include/nfk.h.
extern "C" int nfk_debug_chain_form(int form) {
    const int prev = g_chain_form;
    g_chain_form = form < 0 ? -1 : (form > 1 ? 1 : form);
    return prev;
}

// Diagnostic: the kernel form the last nfk_fused_nsf_chain call launched (-1: none yet).
extern "C" int nfk_debug_last_chain_form() { return g_last_chain_form; }

// ---- the VJP pack (nfk_fused_vjp.hip): records in the 8-coordinate layout,
// then the stream of SB-block sub-records re-cut from them (vjp_dims)
namespace {
__global__ __launch_bounds__(256) void k_vjp_stream(float* pack, Layout L) {
    const VjpDims d = vjp_dims(L.KBH, L.T1, L.K);
    const int64_t total = (int64_t)vjp_nsub(d, L.NCH) * d.SB * 256;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int wl = (int)(g & 255);
        const int64_t blk = g >> 8;
        const int u = (int)(blk / d.SB), b = (int)(blk - (int64_t)u * d.SB);
        int64_t src = -1;  // record block (from the start of the records, o_h1)
        if (u == 0) {
            if (b < L.blk_h1) src = b;
        } else if (u <= d.NP2) {
            const int r = subrec_tile_src(b, L.KBH, L.T1, kVNS, d.HT, (u - 1) * kVNS);
            if (r >= 0) src = L.blk_h1 + r;
        } else {
            const int v = u - 1 - d.NP2, ch = v / d.SPC, w = v - ch * d.SPC;
            int64_t rec = L.blk_h1 + L.blk_h2 + (int64_t)ch * L.blk_chunk;
            int nt = d.KW, t0;
            if (w < d.NPW) {
                t0 = w * kVNS;
            } else if (w < 2 * d.NPW) {
                rec += L.blk_w;
                t0 = (w - d.NPW) * kVNS;
            } else {
                rec += 2 * L.blk_w;
                nt = d.KD;
                t0 = (w - 2 * d.NPW) * kVNS;
            }
            const int r = subrec_tile_src(b, L.KBH, L.T1, kVNS, nt, t0);
            if (r >= 0) src = rec + r;
        }
        pack[L.total + g] = src >= 0 ? pack[L.o_h1 + src * 256 + wl] : 0.0f;
    }
}
}  // namespace

extern "C" int64_t nfk_fused_nsf_vjp_pack_elems(int32_t n_lo, int32_t n_up, int32_t hidden, int32_t K) {
    if (!vjp_ok(n_lo, n_up, hidden, K)) return 0;
    const Layout L = make_layout(n_lo, n_up, hidden, K, 1);
    return L.total + (int64_t)vjp_nsub(vjp_dims(L.KBH, L.T1, K), L.NCH) * vjp_dims(L.KBH, L.T1, K).SB * 256;
}

extern "C" int nfk_fused_nsf_vjp_pack(const float* w0, const float* b0, const float* w2, const float* b2,
                                      const float* w4, const float* b4, int32_t n_lo, int32_t n_up,
                                      int32_t hidden, int32_t K, float* vpack, nfk_stream_t stream) {
    if (!vjp_ok(n_lo, n_up, hidden, K)) return nfk_set_error("nfk_fused_nsf_vjp_pack: shape not supported");
    if (!w0 || !b0 || !w2 || !b2 || !w4 || !b4 || !vpack)
        return nfk_set_error("nfk_fused_nsf_vjp_pack: null pointer");
    PackArgs a{w0, b0, w2, b2, w4, b4, vpack, make_layout(n_lo, n_up, hidden, K, 1)};
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(vpack, 0, 3 * sizeof(float), st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_pack_max, dim3(64), dim3(256), 0, st, a);
    int64_t g = (a.L.total + 255) / 256;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_pack, dim3((unsigned)g), dim3(256), 0, st, a);
    const int64_t n = nfk_fused_nsf_vjp_pack_elems(n_lo, n_up, hidden, K) - a.L.total;
    int64_t gs = (n + 255) / 256;
    if (gs > 8192) gs = 8192;
    hipLaunchKernelGGL(k_vjp_stream, dim3((unsigned)gs), dim3(256), 0, st, vpack, a.L);
    e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

// NSF_CL layers whose conditioner is wider than these kernels take (the
// applications' H = 354, K = 32): nfk_fused_ar.hip's k_fused_cl
bool nfk_cl_ok(int n_lo, int n_up, int hidden, int K);
int64_t nfk_cl_pack_floats(int n_lo, int n_up, int hidden, int K);
int nfk_cl_pack(const float* w0, const float* b0, const float* w2, const float* b2, const float* w4,
                const float* b4, int n_lo, int n_up, int hidden, int K, float* pack, hipStream_t st);
int nfk_cl_launch(const float* x, int64_t ldx, const float* pack, const int32_t* up_in, const int32_t* up_out,
                  int n_up, const int32_t* lo_in, const int32_t* lo_out, int n_lo, int hidden, float* z, int64_t ldz,
                  float* logdet, int mode, int64_t batch, int K, double tail_bound, bool inv, int32_t* status,
                  float* workspace, int64_t workspace_floats, hipStream_t st);
int64_t nfk_cl_workspace(int n_lo, int n_up, int hidden, int K, int64_t batch);

extern "C" int nfk_fused_nsf_supported(int32_t n_lo, int32_t n_up, int32_t hidden, int32_t K) {
    return (pack_ok(n_lo, n_up, hidden, K) || nfk_cl_ok(n_lo, n_up, hidden, K)) ? 1 : 0;
}

extern "C" int64_t nfk_fused_nsf_pack_elems(int32_t n_lo, int32_t n_up, int32_t hidden, int32_t K) {
    if (!pack_ok(n_lo, n_up, hidden, K)) return nfk_cl_pack_floats(n_lo, n_up, hidden, K);
    return pack_floats(n_lo, n_up, hidden, K);
}

extern "C" int nfk_fused_nsf_pack(const float* w0, const float* b0, const float* w2, const float* b2,
                                  const float* w4, const float* b4, int32_t n_lo, int32_t n_up,
                                  int32_t hidden, int32_t K, float* wpack, nfk_stream_t stream) {
    if (!w0 || !b0 || !w2 || !b2 || !w4 || !b4 || !wpack)
        return nfk_set_error("nfk_fused_nsf_pack: null pointer");
    if (!pack_ok(n_lo, n_up, hidden, K)) {
        if (nfk_cl_ok(n_lo, n_up, hidden, K))
            return nfk_cl_pack(w0, b0, w2, b2, w4, b4, n_lo, n_up, hidden, K, wpack, (hipStream_t)stream);
        return nfk_set_error("nfk_fused_nsf_pack: shape not supported");
    }
    PackArgs a{w0, b0, w2, b2, w4, b4, wpack, pack_layout(n_lo, n_up, hidden, K)};
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(wpack, 0, 3 * sizeof(float), st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_pack_max, dim3(64), dim3(256), 0, st, a);
    int64_t g = (pack_floats(n_lo, n_up, hidden, K) + 255) / 256;
    if (g > 8192) g = 8192;
    if (a.L.wide) {
        int s1;
        const int ns = wide_substeps(a.L.KB1, a.L.KBH, K, a.L.NCH, &s1);
        hipLaunchKernelGGL(k_pack_frames, dim3((unsigned)g), dim3(256), 0, st, a, s1, ns,
                           wide_g(a.L.HT, a.L.KBH), wide_g(K / 2, a.L.KBH));
    } else {
        hipLaunchKernelGGL(k_pack, dim3((unsigned)g), dim3(256), 0, st, a);
    }
    e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

namespace {
// kernel arguments shared by nfk_fused_nsf and nfk_fused_nsf_chain
FusedArgs fused_args(const float* x, int64_t ldx, const float* wpack, const int32_t* up_in,
                     const int32_t* up_out, const int32_t* lo_in, const int32_t* lo_out, const Layout& L,
                     float* z, int64_t ldz, float* logdet, int32_t logdet_mode, int64_t batch, int32_t K,
                     double tail_bound, int32_t* status) {
    FusedArgs a;
    a.trace = g_trace;
    a.x = x;
    a.pack = wpack;
    a.up_in = up_in;
    a.up_out = up_out;
    a.lo_in = lo_in;
    a.lo_out = lo_out;
    a.z = z;
    a.logdet = logdet;
    a.status = status;
    a.ldx = ldx;
    a.ldz = ldz;
    a.batch = batch;
    a.n_lo = L.n_lo;
    a.n_up = L.n_up;
    a.KB1 = L.KB1;
    a.NCH = L.NCH;
    a.mode = logdet_mode;
    a.slot_blocks = L.slot_blocks;
    a.xtile = x_tile_floats(L);
    a.xup = x_up_row(L);
    a.blk_h1 = L.blk_h1;
    a.blk_h2 = L.blk_h2;
    a.blk_w = L.blk_w;
    a.blk_d = L.blk_d;
    a.blk_chunk = L.blk_chunk;
    a.o_h1 = (int32_t)L.o_h1;
    a.o_h2 = (int32_t)L.o_h2;
    a.o_w3 = (int32_t)L.o_w3;
    a.packs = nullptr;
    a.cmaps = nullptr;
    a.nlayers = 1;
    a.log_prob = nullptr;
    a.prior_inv_scale = a.prior_c2pi = a.prior_hld = 0.0f;
    a.saves = nullptr;
    a.ld_saves = a.save_stride = 0;
    a.smaps = nullptr;
    {
        // NSF_CL's spline constants (flows.py:236-237 defaults), evaluated like the
        // reference's Python scalars (nfk_make_const), folded for the fixed-point knots
        const NfkSplineConst sc =
            nfk_make_const(K, -tail_bound, tail_bound, -tail_bound, tail_bound, 1, 1e-3, 1e-3, 1e-3);
        const float two30 = 1073741824.0f;
        a.c.lo = sc.lo;
        a.c.hi = sc.hi;
        a.c.sp30 = sc.span / two30;
        a.c.inv30 = two30 / sc.span;
        a.c.fb30 = sc.fw * two30;
        a.c.mb30 = sc.min_w * two30;
        a.c.m2b = sc.m2b;
        a.c.min_d = sc.min_d;
        a.c.d_edge = sc.d_edge;
    }
    return a;
}
}  // namespace

extern "C" int64_t nfk_fused_nsf_workspace(int32_t n_lo, int32_t n_up, int32_t hidden, int32_t K, int64_t batch,
                                           int32_t inverse) {
    (void)inverse;
    if (shape_ok(n_lo, n_up, hidden, K) || wide_ok(n_lo, n_up, hidden, K)) return 0;
    return nfk_cl_workspace(n_lo, n_up, hidden, K, batch);
}

extern "C" int nfk_fused_nsf_ws(const float* x, int64_t ldx, const float* wpack, const int32_t* up_in,
                                const int32_t* up_out, int32_t n_up, const int32_t* lo_in, const int32_t* lo_out,
                                int32_t n_lo, int32_t hidden, float* z, int64_t ldz, float* logdet,
                                int32_t logdet_mode, int64_t batch, int32_t K, double tail_bound, int32_t inverse,
                                int32_t* status, float* workspace, int64_t workspace_floats, nfk_stream_t stream);

extern "C" int nfk_fused_nsf(const float* x, int64_t ldx, const float* wpack, const int32_t* up_in,
                             const int32_t* up_out, int32_t n_up, const int32_t* lo_in,
                             const int32_t* lo_out, int32_t n_lo, int32_t hidden, float* z,
                             int64_t ldz, float* logdet, int32_t logdet_mode, int64_t batch,
                             int32_t K, double tail_bound, int32_t inverse, int32_t* status,
                             nfk_stream_t stream) {
    return nfk_fused_nsf_ws(x, ldx, wpack, up_in, up_out, n_up, lo_in, lo_out, n_lo, hidden, z, ldz, logdet,
                            logdet_mode, batch, K, tail_bound, inverse, status, nullptr, 0, stream);
}

extern "C" int nfk_fused_nsf_ws(const float* x, int64_t ldx, const float* wpack, const int32_t* up_in,
                                const int32_t* up_out, int32_t n_up, const int32_t* lo_in, const int32_t* lo_out,
                                int32_t n_lo, int32_t hidden, float* z, int64_t ldz, float* logdet,
                                int32_t logdet_mode, int64_t batch, int32_t K, double tail_bound, int32_t inverse,
                                int32_t* status, float* workspace, int64_t workspace_floats, nfk_stream_t stream) {
    const bool narrow = shape_ok(n_lo, n_up, hidden, K);
    const bool cl = !narrow && !wide_ok(n_lo, n_up, hidden, K) && nfk_cl_ok(n_lo, n_up, hidden, K);
    if (!narrow && !cl && !wide_ok(n_lo, n_up, hidden, K)) return nfk_set_error("nfk_fused_nsf: shape not supported");
    if (batch < 0) return nfk_set_error("nfk_fused_nsf: bad batch");
    if (batch == 0) return 0;
    if (!x || !wpack || !up_in || !up_out || !lo_in || !lo_out || !z)
        return nfk_set_error("nfk_fused_nsf: null pointer");
    if (logdet_mode != 0 && !logdet) return nfk_set_error("nfk_fused_nsf: null logdet");
    if (cl)
        return nfk_cl_launch(x, ldx, wpack, up_in, up_out, n_up, lo_in, lo_out, n_lo, hidden, z, ldz, logdet,
                             logdet_mode, batch, K, tail_bound, inverse != 0, status, workspace, workspace_floats,
                             (hipStream_t)stream);
    const Layout L = pack_layout(n_lo, n_up, hidden, K);
    FusedArgs a = fused_args(x, ldx, wpack, up_in, up_out, lo_in, lo_out, L, z, ldz, logdet, logdet_mode, batch,
                             K, tail_bound, status);
    hipStream_t st = (hipStream_t)stream;
    const bool inv = inverse != 0;
    if (!narrow) return launch_wide(a, L, K, inv, st);
    // split form (sub-records, three workgroups per CU) where it fits;
    // NFK_FUSED_SPLIT=0 in the environment or nfk_debug_fused_form(0) selects
    // whole records (A/B runs, tests of both forms)
    static const bool split_env = [] {
        const char* e = std::getenv("NFK_FUSED_SPLIT");
        return !(e != nullptr && e[0] == '0');
    }();
    const bool aligned16 = ((uintptr_t)x % 16) == 0 && ((uintptr_t)z % 16) == 0 && ldx % 4 == 0 && ldz % 4 == 0;
    const bool split = (g_form < 0 ? split_env : g_form == 1) && split_ok(L) && aligned16;
    if (split) {
        a.slot_blocks = split_slot_blocks(L);
        a.xtile = 16 * (n_lo + n_up + 1);
    }
    const size_t lds = split ? lds_bytes_split(L) : lds_bytes(L);
#define DISPATCH(h, t, k) \
    if (L.KBH == h && L.T1 == t && K == k) return launch_fused<h, t, k>(a, lds, inv, split, false, st);
#define DISPATCH_KB(h, t) NFK_FUSED_K(DISPATCH, h, t)
    NFK_FUSED_KB(DISPATCH_KB)
#undef DISPATCH_KB
#undef DISPATCH
    return nfk_set_error("nfk_fused_nsf: no kernel instance");
}

extern "C" int nfk_fused_nsf_chain_max(int32_t n_lo, int32_t n_up, int32_t hidden, int32_t K) {
    if (!shape_ok(n_lo, n_up, hidden, K)) return 0;
    return chain_max_layers(make_layout(n_lo, n_up, hidden, K));
}

extern "C" int nfk_fused_nsf_chain(const float* x, int64_t ldx, const float* const* wpacks,
                                   const int32_t* cmaps, int32_t nlayers, int32_t n_lo, int32_t n_up,
                                   int32_t hidden, float* z, int64_t ldz, float* logdet,
                                   int32_t logdet_mode, int64_t batch, int32_t K, double tail_bound,
                                   int32_t inverse, int32_t* status, float* log_prob, float prior_scale,
                                   float prior_half_log_det, nfk_stream_t stream) {
    if (!shape_ok(n_lo, n_up, hidden, K)) return nfk_set_error("nfk_fused_nsf_chain: shape not supported");
    const Layout L = make_layout(n_lo, n_up, hidden, K);
    const int nmax = chain_max_layers(L);
    if (nlayers < 1 || nlayers > nmax) return nfk_set_error("nfk_fused_nsf_chain: bad layer count");
    if (batch < 0) return nfk_set_error("nfk_fused_nsf_chain: bad batch");
    if (batch == 0) return 0;
    if (!x || !wpacks || !cmaps || (!z && !log_prob)) return nfk_set_error("nfk_fused_nsf_chain: null pointer");
    if (log_prob && !(prior_scale > 0.0f)) return nfk_set_error("nfk_fused_nsf_chain: bad prior scale");
    if (logdet_mode != 0 && !logdet) return nfk_set_error("nfk_fused_nsf_chain: null logdet");
    if (((uintptr_t)x % 16) != 0 || ((uintptr_t)z % 16) != 0 || ldx % 4 != 0 || (z && ldz % 4 != 0))
        return nfk_set_error("nfk_fused_nsf_chain: x and z rows must be 16-byte aligned");
    if (ldx < n_lo + n_up || (z && ldz < n_lo + n_up))
        return nfk_set_error("nfk_fused_nsf_chain: ldx and ldz must be >= n_lo + n_up");
    FusedArgs a = fused_args(x, ldx, nullptr, nullptr, nullptr, nullptr, nullptr, L, z, ldz, logdet, logdet_mode,
                             batch, K, tail_bound, status);
    a.slot_blocks = split_slot_blocks(L);
    a.xtile = 16 * (n_lo + n_up + 1);
    a.packs = wpacks;
    a.cmaps = cmaps;
    a.nlayers = nlayers;
    if (log_prob) {  // the constants of nfk_normal_logprob
        a.log_prob = log_prob;
        a.prior_inv_scale = 1.0f / prior_scale;
        a.prior_c2pi = (float)((n_lo + n_up) * std::log(2.0 * M_PI));
        a.prior_hld = prior_half_log_det;
    }
    hipStream_t st = (hipStream_t)stream;
    const bool inv = inverse != 0;
    // kernel forms: 1 = two 16-sample tiles per wave (nfk_fused_chain2.hip;
    // c3: 5.83-5.84 vs 6.02 ms per 2^20 log_prob, 0.805 vs 0.832 ms at 2^17
    // against form 0, profiles/r3c_chain2_ab.txt) where instanced; 0 = one
    // tile.  NFK_CHAIN_FORM in the environment or nfk_debug_chain_form
    // overrides the default.  (A 32x32x16 form measured 1-4 % slower once
    // both had branch-free epilogue reads: DESIGN.md section 6.)
    static const int form_env = [] {
        const char* e = std::getenv("NFK_CHAIN_FORM");
        return (e != nullptr && e[0] >= '0' && e[0] <= '1') ? e[0] - '0' : kChainFormDefault;
    }();
    const int form = g_chain_form < 0 ? form_env : g_chain_form;
    if (form >= 1 && chain2_ok(L, K, nlayers)) {
        const int rc = launch_chain2(a, L, K, inv, st);
        g_last_chain_form = 1;
        if (rc >= 0) return rc;
    }
    g_last_chain_form = 0;
    const size_t lds = lds_bytes_chain(L, nlayers);
#define DISPATCH(h, t, k) \
    if (L.KBH == h && L.T1 == t && K == k) return launch_fused<h, t, k>(a, lds, inv, true, true, st);
#define DISPATCH_KB(h, t) NFK_FUSED_K(DISPATCH, h, t)
    NFK_FUSED_KB(DISPATCH_KB)
#undef DISPATCH_KB
#undef DISPATCH
    return nfk_set_error("nfk_fused_nsf_chain: no kernel instance");
}

extern "C" int nfk_fused_nsf_chain_saved_ok(int32_t n_lo, int32_t n_up, int32_t hidden, int32_t K,
                                            int32_t nlayers) {
    if (!shape_ok(n_lo, n_up, hidden, K) || nlayers < 2) return 0;
    const Layout L = make_layout(n_lo, n_up, hidden, K);
    return nlayers <= chain_max_layers(L) && chain2_ok(L, K, nlayers, true) ? 1 : 0;
}

extern "C" int nfk_fused_nsf_chain_saved(const float* x, int64_t ldx, const float* const* wpacks,
                                         const int32_t* cmaps, int32_t nlayers, int32_t n_lo, int32_t n_up,
                                         int32_t hidden, float* z, int64_t ldz, float* logdet,
                                         int32_t logdet_mode, int64_t batch, int32_t K, double tail_bound,
                                         int32_t* status, float* saves, int64_t ld_saves, int64_t save_stride,
                                         const int32_t* smaps, nfk_stream_t stream) {
    if (!nfk_fused_nsf_chain_saved_ok(n_lo, n_up, hidden, K, nlayers))
        return nfk_set_error("nfk_fused_nsf_chain_saved: shape or layer count not supported");
    if (batch < 0) return nfk_set_error("nfk_fused_nsf_chain_saved: bad batch");
    if (batch == 0) return 0;
    if (!x || !wpacks || !cmaps || !z || !saves || !smaps)
        return nfk_set_error("nfk_fused_nsf_chain_saved: null pointer");
    if (logdet_mode != 0 && !logdet) return nfk_set_error("nfk_fused_nsf_chain_saved: null logdet");
    const int D = n_lo + n_up;
    if (((uintptr_t)x % 16) != 0 || ((uintptr_t)z % 16) != 0 || ((uintptr_t)saves % 16) != 0 || ldx % 4 != 0 ||
        ldz % 4 != 0 || ld_saves % 4 != 0 || save_stride % 4 != 0 || ld_saves < D || save_stride < batch * ld_saves)
        return nfk_set_error("nfk_fused_nsf_chain_saved: x, z and saves rows must be 16-byte aligned");
    if (ldx < D || ldz < D) return nfk_set_error("nfk_fused_nsf_chain_saved: ldx and ldz must be >= n_lo + n_up");
    const Layout L = make_layout(n_lo, n_up, hidden, K);
    FusedArgs a = fused_args(x, ldx, nullptr, nullptr, nullptr, nullptr, nullptr, L, z, ldz, logdet, logdet_mode,
                             batch, K, tail_bound, status);
    a.slot_blocks = split_slot_blocks(L);
    a.xtile = 16 * D + 16;
    a.packs = wpacks;
    a.cmaps = cmaps;
    a.nlayers = nlayers;
    a.saves = saves;
    a.ld_saves = ld_saves;
    a.save_stride = save_stride;
    a.smaps = smaps;
    const int rc = launch_chain2(a, L, K, false, (hipStream_t)stream);
    return rc >= 0 ? rc : nfk_set_error("nfk_fused_nsf_chain_saved: no kernel instance");
}
