// nfk_ar_seqinv.hip -- the NSF_AR inverse (nf/flows.py:193-209) for the layers
// whose inverse the fused register form cannot hold: Polymer.yaml's 2,048
// coordinates (applications/input/Polymer.yaml:8-9, 17-18; sampled by the
// applications' sample() calls, nf/models.py:31-35).
//
// The inverse is sequential: conditioner i reads the trig features of the
// coordinates already inverted (x[:, :i], flows.py:201), so coordinate i waits
// for i - 1.  ONE launch per coordinate, issued from C++ (no host round trip
// and no Python between them), k_sq_step:
//
//   workgroups 0 .. M-1     finish conditioner i, one row each: its layer-1
//                           chunks summed in order, plus the products of x_(i-1)'s
//                           two features, + b1, tanh, layer 2, tanh, the output
//                           layer (95 logits), the spline's inverse on one
//                           wave (sq_spline_inv: the reference's 2B softmax /
//                           softplus, then RQS, utils.py:27-152), x[m, i], the
//                           row's log|det| in column order (flows.py:208), the
//                           status word of column i, cos / sin (pi x_i / B)
//   workgroups M ..         layer 1 of conditioner i + 1 over its features in
//                           64-feature chunks, all but x_i's two (which the
//                           first group is computing), two workgroups per chunk
//                           (the halves of the units): [M, 64] x [64, H / 2]
//                           register tiles, fp32 partial sums (double-buffered
//                           by conditioner parity)
//   the last 8              conditioner i + 1's W2, W3, biases and two W1
//                           columns read into each XCD's L2 for the next launch
//
// The conditioners' nn.Linear weights are read in place (fp32; a host table of
// their device pointers, passed to each launch as arguments), and the
// arithmetic is fp32 FMA throughout: the inverse is latency-bound (2,048
// dependent launches per layer at Polymer's shape, ~7.3 us each), not
// bandwidth- or FLOP-bound, and every weight is read once per layer (1.68 GB
// at Polymer, 0.2 ms of HBM time).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>

#include "../../include/nfk.h"
#include "nfk_spline.h"

int nfk_set_error(const char* msg);  // nfk_kernels.hip
NfkSplineConst nfk_make_const(int K, double left, double right, double bottom, double top, int tails, double min_w,
                              double min_h, double min_d);

namespace {

constexpr int kSqFC = 64;        // layer-1 features per chunk workgroup
constexpr int kSqThreads = 256;  // both kernels
constexpr int kSqMaxRows = 64;   // rows per pass
constexpr int kSqMaxH = 128;     // hidden width (a chunk workgroup takes half of the units)

typedef float sq_f4 __attribute__((ext_vector_type(4)));  // (HIP's float4 struct arrays went to scratch)
typedef float sq_f2 __attribute__((ext_vector_type(2)));
// The conditioners' weights come through a device table of pointers, which the
// compiler cannot place in an address space: their loads were FLAT ones (which
// every LDS wait also waits for).  Each such pointer is cast to global.
typedef __attribute__((address_space(1))) const float sq_gf;
typedef __attribute__((address_space(1))) const sq_f4 sq_gf4;
typedef __attribute__((address_space(1))) const sq_f2 sq_gf2;
__device__ __forceinline__ sq_gf* sq_glb(const float* p) { return (sq_gf*)p; }

// one conditioner's nn.Linear tensors: W1 [H, 2i], b1, W2 [H, H], b2, W3 [P, H], b3
struct SqCond {
    const float *W1, *b1, *W2, *b2, *W3, *b3;
};

struct SqArgs {
    const float* init;      // init_param [P]
    const float* z;         // this pass's rows of the layer input
    int64_t ldz;
    float* x;               // ... of the output
    int64_t ldx;
    float* feat;            // [2][M][dim]: cos, sin (pi x / B) of the inverted coordinates
    float* part;            // [2][M][chunks][H] layer-1 partial sums (by conditioner parity)
    float* ldacc;           // [M] the rows' log|det| so far (column order)
    float* logdet;          // [M] (this pass's rows) or null
    int32_t* status;        // [dim] or null
    int mode, dim, H, M, nchmax;
    float pi, bnd;
    NfkSplineConst c;
    unsigned long long* tdbg;  // diagnostic phase clocks (nfk_debug_sq_timing), normally null
    float* sink;               // [kSqThreads] workspace floats the prefetch workgroups' sums feed (never read)
};

// diagnostic: thread 0 of row 0's finish and of the first chunk workgroup stamp
// the shader clock at their phase boundaries, [dim][12] per pass
__device__ __forceinline__ void sq_stamp(const SqArgs& a, int i, int slot) {
    if (a.tdbg != nullptr && threadIdx.x == 0) a.tdbg[(int64_t)i * 12 + slot] = __builtin_readcyclecounter();
}

// LDS of a k_sq_step workgroup: the finish part's (h1, h2, the logits) or the
// layer-1 part's (64 features x 64 units of weights, 64 features x 64 rows),
// the larger
inline size_t sq_fin_floats(int H, int K) {
    (void)H;
    return (size_t)(2 * 128 + 3 * K - 1);  // h1, h2 (kSqMaxH each), logits
}
// chunk workgroups' LDS strides: weights [unit][feature] rows kSqWS apart (odd:
// the staging stores and the GEMM's per-unit reads both conflict-free), the
// rows' features [feature][row] kSqFS apart (16-byte aligned row quads)
constexpr int kSqWS = kSqFC + 1;
constexpr int kSqFS = kSqMaxRows + 4;
inline size_t sq_lds(int nch, int H, int K) {
    const size_t l1 = (size_t)(kSqMaxH / 2) * kSqWS + (size_t)kSqFC * kSqFS;
    const size_t f = sq_fin_floats(H, K);
    (void)nch;
    return (f > l1 ? f : l1) * sizeof(float);
}

// layer 1 of conditioner j over features f0 .. f0 + 63 (chunk c = cc / 2) for
// one half of its units (cc % 2), WITHOUT the two features of coordinate j - 1
// (cos at f = j - 1, sin at f = 2j - 1: the finish of column j - 1 runs in the
// same launch and writes them; the finish of conditioner j adds their products
// itself).  Every operand is requested before any is stored (one memory round
// trip), through LDS as ws [unit][feature] and fs [feature][row]; each thread a
// 4-row x 2-unit tile
__device__ void sq_l1_chunk(const SqArgs& a, const float* W1j, int j, int cc, float* lds) {
    float* ws = lds;                                      // [kSqMaxH / 2][kSqWS]
    float* fs = lds + (kSqMaxH / 2) * kSqWS;              // [kSqFC][kSqFS]
    const int c = cc >> 1, F = 2 * j, f0 = c * kSqFC, nf = F - f0 < kSqFC ? F - f0 : kSqFC;
    const int H = a.H, M = a.M, HH = ((H + 3) / 4) * 2;  // (units per half: even)
    const int u_lo = (cc & 1) * HH, nu = H - u_lo < HH ? H - u_lo : HH;
    if (cc == 0) sq_stamp(a, j - 1, 8);
    // (feature pairs: F = 2j is even, so every row segment is 8-byte aligned;
    // 32 pairs per unit row, consecutive threads along one row.  Branch-free
    // loads: a clamped index, then a select -- loads under divergent branches
    // had each been followed by a wait)
    constexpr int FC2 = kSqFC / 2, UW = (kSqMaxH / 2) * FC2 / kSqThreads, UF = kSqMaxRows * kSqFC / kSqThreads;
    sq_gf2* W1p = reinterpret_cast<sq_gf2*>(sq_glb(W1j));
    sq_f2 wv[UW];
    float fv[UF];
#pragma unroll
    for (int u = 0; u < UW; ++u) {
        const int e = threadIdx.x + u * kSqThreads, h = e / FC2, f = 2 * (e - h * FC2);
        const bool ok = h < nu && f < nf;
        wv[u] = W1p[ok ? ((int64_t)(u_lo + h) * F + f0 + f) >> 1 : 0];
        wv[u] = ok ? wv[u] : sq_f2{0.0f, 0.0f};
    }
    // feature f of conditioner j: cos(pi x_f / B) for f < j, sin(pi x_(f-j) / B)
    // above (trig_transform's cat, flows.py:172-173)
#pragma unroll
    for (int u = 0; u < UF; ++u) {
        const int e = threadIdx.x + u * kSqThreads, m = e / kSqFC, f = e - m * kSqFC, g = f0 + f;
        const bool ok = m < M && f < nf && g != j - 1 && g != 2 * j - 1;
        const int64_t idx = g < j ? (int64_t)m * a.dim + g : ((int64_t)M + m) * a.dim + (g - j);
        fv[u] = a.feat[ok ? idx : 0];
        fv[u] = ok ? fv[u] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < UW; ++u) {
        const int e = threadIdx.x + u * kSqThreads, h = e / FC2, f = 2 * (e - h * FC2);
        ws[h * kSqWS + f] = wv[u].x;
        ws[h * kSqWS + f + 1] = wv[u].y;
    }
#pragma unroll
    for (int u = 0; u < UF; ++u) {
        const int e = threadIdx.x + u * kSqThreads, m = e / kSqFC, f = e - m * kSqFC;
        fs[f * kSqFS + m] = fv[u];
    }
    __syncthreads();
    if (cc == 0) sq_stamp(a, j - 1, 9);
    float* part = a.part + (int64_t)(j & 1) * M * a.nchmax * H;
    const int HT = (nu + 1) / 2, MT4 = (M + 3) / 4;
    typedef float f4v __attribute__((ext_vector_type(4)));
    for (int t = threadIdx.x; t < HT * MT4; t += kSqThreads) {
        const int u0 = 2 * (t % HT), m0 = 4 * (t / HT);
        const float* w0 = ws + u0 * kSqWS;
        const float* w1 = w0 + kSqWS;  // (u0 + 1 <= HH - 1 < kSqMaxH / 2: inside the buffer)
        float acc[4][2];
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r][0] = acc[r][1] = 0.0f;
#pragma unroll 8
        for (int f = 0; f < nf; ++f) {
            const f4v x = *reinterpret_cast<const f4v*>(fs + f * kSqFS + m0);
            const float wa = w0[f], wb = w1[f];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                acc[r][0] = __builtin_fmaf(x[r], wa, acc[r][0]);
                acc[r][1] = __builtin_fmaf(x[r], wb, acc[r][1]);
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int q = 0; q < 2; ++q)
                if (m0 + r < M && u0 + q < nu)
                    part[((int64_t)(m0 + r) * a.nchmax + c) * H + u_lo + u0 + q] = acc[r][q];
    }
    if (cc == 0) sq_stamp(a, j - 1, 10);
}

// the operands the next launch's finish stages from the conditioners' weights
// (conditioner j: W2, W3, the biases, x_(j-1)'s two columns of W1) read into
// this XCD's L2 (one such workgroup per XCD: 8 consecutive workgroups), their
// sum fed to a store that never happens so the loads are kept
__device__ void sq_prefetch(const SqArgs& a, const SqCond& w, int j, int K3) {
    const int H = a.H, P = K3;
    sq_gf *W1 = sq_glb(w.W1), *W2 = sq_glb(w.W2), *W3 = sq_glb(w.W3);
    float acc = 0.0f;
    const int n2 = H * H, n3 = P * H;
    // one 4-byte load per 64-byte segment is enough to bring the line in
    for (int e = threadIdx.x * 16; e < n2; e += kSqThreads * 16) acc += W2[e];
    for (int e = threadIdx.x * 16; e < n3; e += kSqThreads * 16) acc += W3[e];
    const int h = threadIdx.x < H ? threadIdx.x : 0, p = threadIdx.x < P ? threadIdx.x : 0;
    sq_gf* wr = W1 + (int64_t)h * 2 * j;
    acc += wr[j - 1] + wr[2 * j - 1] + sq_glb(w.b1)[h] + sq_glb(w.b2)[h] + sq_glb(w.b3)[p];
    if (acc == 1.0e-30f) a.sink[threadIdx.x] = acc;
}

// sums over lane pairs / 16-lane groups by DPP moves (no LDS round trip, as
// __shfl_xor's ds_bpermute has): xor 1, xor 2 (quad permutes), then the
// half-row and row mirrors, which swap the already-equal quads / halves; each
// step adds a lane's value and its partner's, so every lane ends with the
// same sum
template <int CTRL>
__device__ __forceinline__ float sq_dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float sq_sum2(float v) { return v + sq_dpp<0xB1>(v); }
// the same over a 32-lane half: the rows by DPP, then one swap of the rows
__device__ __forceinline__ float sq_max32(float v) {
    v = fmaxf(v, sq_dpp<0xB1>(v));
    v = fmaxf(v, sq_dpp<0x4E>(v));
    v = fmaxf(v, sq_dpp<0x141>(v));
    v = fmaxf(v, sq_dpp<0x140>(v));
    return fmaxf(v, __shfl_xor(v, 16, 32));
}
__device__ __forceinline__ float sq_sum16(float v);
__device__ __forceinline__ float sq_sum32(float v) {
    v = sq_sum16(v);
    return v + __shfl_xor(v, 16, 32);
}
// inclusive prefix sum of ints over each 32-lane half: row_shr 1, 2, 4, 8
// within each 16-lane row (lanes shifted in from outside the row add 0), then
// row_bcast:15 carries row 0's (row 2's) total into row 1 (row 3)
template <int CTRL, int ROWS>
__device__ __forceinline__ int sq_idpp(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWS, 0xF, true);
}
__device__ __forceinline__ int sq_scan32(int v) {
    v += sq_idpp<0x111, 0xF>(v);
    v += sq_idpp<0x112, 0xF>(v);
    v += sq_idpp<0x114, 0xF>(v);
    v += sq_idpp<0x118, 0xF>(v);
    return v + __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
}
__device__ __forceinline__ float sq_sum16(float v) {
    v += sq_dpp<0xB1>(v);   // quad_perm [1, 0, 3, 2]
    v += sq_dpp<0x4E>(v);   // quad_perm [2, 3, 0, 1]
    v += sq_dpp<0x141>(v);  // row_half_mirror
    return v + sq_dpp<0x140>(v);  // row_mirror
}

// The spline's inverse for one element on one wave (nfk_rqs_element_lean's
// algorithm, utils.py:58-152 with the 2B softmax / softplus of flows.py:206-207,
// spread over lanes): lanes 0-31 take the K width logits, 32-63 the K height
// logits; max, the two softmax sums (DPP within 16-lane rows, then one row
// swap: every lane the same sum) and the integer knot prefixes (a DPP lane
// scan: exact, so the knots are those of the sequential prefix) run in
// parallel, the bin is a ballot count, and every lane then evaluates the same
// bin.  Every lane of the wave must call it.
template <int K>
__device__ __forceinline__ void sq_spline_inv(const float* lg, float x, const NfkSplineConst& c, float& out,
                                              float& lad, bool& inside, bool& neg_disc) {
    static_assert(K >= 2 && K <= 32, "sq_spline_inv: one logit per lane of a 32-lane half");
    const int lane = threadIdx.x & 63, hb = lane >> 5, p = lane & 31;
    const bool act = p < K;
    inside = !c.tails || ((x >= c.lo) && (x <= c.hi));
    neg_disc = false;
    const float two30 = 1073741824.0f;
    const float sp30 = c.span * (1.0f / two30), inv30 = two30 / c.span;
    const float fb30 = c.fw * two30, mb30 = c.min_w * two30;
    const float raw = lg[hb * K + (act ? p : 0)];
    const float mx = sq_max32(act ? raw : -INFINITY);
    const float mL = mx * kL2E;
    float e = act ? __builtin_amdgcn_exp2f(__builtin_fmaf(raw, kL2E, -mL)) : 0.0f;
    const float s1 = sq_sum32(e);
    const float q = c.m2b * __builtin_amdgcn_rcpf(s1);
    e = act ? __builtin_amdgcn_exp2f(__builtin_fmaf(e, q, -c.m2b)) : 0.0f;
    const float s2 = sq_sum32(e);
    const float f30 = fb30 * __builtin_amdgcn_rcpf(s2);
    const int v = p < K - 1 ? (int)__builtin_fmaf(e, f30, mb30) : 0;
    const int pre = sq_scan32(v) - v;  // knot p's integer position (pre[0] = 0)
    // (wave-uniform values by v_readlane: no LDS round trips)
    const float s2w = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, s2), 0));
    const float s2h = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, s2), 32));
    // the bin: how many inner height knots x has passed
    const int xi = __float2int_rd(__builtin_fmaf(x, inv30, -c.lo * inv30));
    const int k = __popcll(__ballot(hb == 1 && p >= 1 && p < K && xi >= pre));
    const int k1 = k + 1 < K ? k + 1 : 0;
    const int pw0 = __builtin_amdgcn_readlane(pre, k), pw1 = __builtin_amdgcn_readlane(pre, k1);
    const int ph0 = __builtin_amdgcn_readlane(pre, 32 + k), ph1 = __builtin_amdgcn_readlane(pre, 32 + k1);
    const float low = __builtin_fmaf(s2w, 0.0f, c.lo), loh = __builtin_fmaf(s2h, 0.0f, c.lo);
    const float cw_k = __builtin_fmaf(sp30, (float)pw0, low);
    const float w_k = ((k == K - 1) ? c.hi : __builtin_fmaf(sp30, (float)pw1, low)) - cw_k;
    const float ch_k = __builtin_fmaf(sp30, (float)ph0, loh);
    const float h_k = ((k == K - 1) ? c.hi : __builtin_fmaf(sp30, (float)ph1, loh)) - ch_k;
    // padded derivative index j + 1 holds logit j (utils.py:36-39)
    const float raw_k = lg[2 * K + (k >= 1 ? k - 1 : 0)], raw_k1 = lg[2 * K + (k < K - 1 ? k : 0)];
    const float d_k = (k == 0) ? c.d_edge : nfk_deriv_lean(raw_k, c.min_d);
    const float d_k1 = (k == K - 1) ? c.d_edge : nfk_deriv_lean(raw_k1, c.min_d);
    const float rw = nfk_rcp_fast(w_k);
    const float delta = h_k * rw;
    const float gap = (d_k + d_k1) - 2.0f * delta;
    const float y = x - ch_k;
    const float qa = y * gap + h_k * (delta - d_k);
    const float qb = h_k * d_k - y * gap;
    const float qc = (-delta) * y;
    const float disc = qb * qb - (4.0f * qa) * qc;
    neg_disc = inside && !(disc >= 0.0f);
    const float th = nfk_div_fast(2.0f * qc, -qb - sqrtf(disc));
    out = th * w_k + cw_k;
    const float t1mt = th * (1.0f - th);
    const float den = delta + gap * t1mt;
    const float omt = 1.0f - th;
    const float dnum = (delta * delta) * ((d_k1 * (th * th) + (2.0f * delta) * t1mt) + d_k * (omt * omt));
    const float l = (__builtin_amdgcn_logf(dnum) - 2.0f * __builtin_amdgcn_logf(den)) * kLN2;
    lad = inside ? -l : 0.0f;
    out = inside ? out : x;
}

// the rest of conditioner i for ONE row m: its layer-1 chunk sums, + the
// products of coordinate i - 1's two features (left out of the chunks), + b1,
// tanh, layer 2, tanh, the output layer, the spline's inverse, x[m, i], the
// row's log|det|, the status word, cos / sin of x[m, i].
// Register form, every operand loaded once at the start (one round trip), only
// the activations through LDS:
//   layer 1   lanes 2o, 2o + 1: unit o, the row's chunk sums c = half, half + 2,
//             ... (consecutive lanes on consecutive units: coalesced), the
//             halves added by a lane swap (the same sum on both lanes)
//   layers    16-lane groups g = tid / 16: outputs o = g + 16 p (pass p), lane
//   2 and 3   l of the group on inputs 4l .. 4l + 3 and 64 + 4l .. 67 + 4l, so a
//             group reads 256 contiguous bytes of a weight row per load; the
//             16 lanes' dot products added by DPP moves (sq_sum16: the same
//             sum on every lane), lane p then finishing output g + 16 p
template <int K>
__device__ void sq_finish(const SqArgs& a, const SqCond& wt, int i, int nch, int m, float* lds) {
    constexpr int P = 3 * K - 1;
    constexpr int NP2 = kSqMaxH / 16, NP3 = (P + 15) / 16;  // passes of layers 2, 3
    constexpr int CQ = 32;                                  // partial sums per lane per round
    static_assert(kSqMaxH <= 128 && kSqThreads == 256, "sq_finish: 16 groups of 16 lanes, inputs 4l and 64 + 4l");
    typedef sq_f4 f4v;
    const int H = a.H, tid = threadIdx.x, ho = tid >> 1, half = tid & 1, g = tid >> 4, l = tid & 15;
    const int HA = (H + 3) & ~3;
    float* h1 = lds;         // [128] (zero past H: the layer reads run to 128)
    float* h2 = h1 + 128;    // [128]
    float* lg = h2 + 128;    // [P]
    if (m == 0) sq_stamp(a, i, 0);
    float zv = 0.0f, ldprev = 0.0f;
    if (tid < 64) {  // (the spline's wave)
        zv = a.z[(int64_t)m * a.ldz + i];
        ldprev = i == 0 ? 0.0f : a.ldacc[m];
    }
    if (i == 0) {
        // coordinate 0: init_param, the same logits for every row (flows.py:196-199)
        for (int p = tid; p < P; p += kSqThreads) lg[p] = a.init[p];
    } else {
        // every load issued before any is waited for; indices clamped (no branches)
        const bool al = (H & 3) == 0 &&
                        ((reinterpret_cast<uintptr_t>(wt.W2) | reinterpret_cast<uintptr_t>(wt.W3)) & 15) == 0;
        sq_gf *W2 = sq_glb(wt.W2), *W3 = sq_glb(wt.W3);
        f4v w2r[NP2][2], w3r[NP3][2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int k = 64 * j + 4 * l, kc = k < H ? k : 0;
#pragma unroll
            for (int p = 0; p < NP2; ++p) {
                const int o = g + 16 * p, oc = o < H ? o : 0;
                if (al) {
                    w2r[p][j] = *reinterpret_cast<sq_gf4*>(W2 + (int64_t)oc * H + kc);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) w2r[p][j][e] = W2[(int64_t)oc * H + (k + e < H ? k + e : 0)];
                }
            }
#pragma unroll
            for (int p = 0; p < NP3; ++p) {
                const int o = g + 16 * p, oc = o < P ? o : 0;
                if (al) {
                    w3r[p][j] = *reinterpret_cast<sq_gf4*>(W3 + (int64_t)oc * H + kc);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) w3r[p][j][e] = W3[(int64_t)oc * H + (k + e < H ? k + e : 0)];
                }
            }
        }
        const int o1 = ho < H ? ho : 0;
        sq_gf* pp = sq_glb(a.part + ((int64_t)(i & 1) * a.M + m) * a.nchmax * H + o1);
        float pv[CQ];
#pragma unroll
        for (int u = 0; u < CQ; ++u) {
            const int c = half + 2 * u;
            pv[u] = pp[(int64_t)(c < nch ? c : 0) * H];
        }
        sq_gf* w1r = sq_glb(wt.W1) + (int64_t)o1 * 2 * i;
        const float wa = w1r[i - 1], wb = w1r[2 * i - 1];
        const float cp = a.feat[(int64_t)m * a.dim + i - 1];
        const float sp = a.feat[((int64_t)a.M + m) * a.dim + i - 1];
        // biases: b1 of unit ho (layer 1); b2, b3 of output g + 16 l (lane l finishes pass l)
        const int o2 = g + 16 * l;
        const float bias1 = sq_glb(wt.b1)[o1], bias2 = sq_glb(wt.b2)[o2 < H ? o2 : 0];
        const float bias3 = sq_glb(wt.b3)[o2 < P ? o2 : 0];
        if (tid >= H && tid < 128) h1[tid] = h2[tid] = 0.0f;
        // (no masks: past a row's end the clamped loads re-read the same row's
        // first weights, finite wherever the row's own output is, and meet
        // h1 / h2's zero padding -- fma(0, w, t) = t exactly; the rows past
        // the last output are computed and dropped.  Masking the weights had
        // cost 112 selects per lane on the critical path.)
        if (m == 0) sq_stamp(a, i, 1);
        // layer 1: the chunk sums in chunk order within each lane's half
        float s = 0.0f;
#pragma unroll
        for (int u = 0; u < CQ; ++u)
            if (half + 2 * u < nch) s += pv[u];
        for (int c0 = half + 2 * CQ; c0 < nch; c0 += 2 * CQ) {  // (more than 2 CQ chunks: dim > 2049)
#pragma unroll
            for (int u = 0; u < CQ; ++u) {
                const int c = c0 + 2 * u;
                pv[u] = pp[(int64_t)(c < nch ? c : 0) * H];
            }
#pragma unroll
            for (int u = 0; u < CQ; ++u)
                if (c0 + 2 * u < nch) s += pv[u];
        }
        s = sq_sum2(s);
        s = __builtin_fmaf(cp, wa, s);
        s = __builtin_fmaf(sp, wb, s);
        if (half == 0 && ho < H) h1[ho] = tanhf(s + bias1);
        __syncthreads();
        if (m == 0) sq_stamp(a, i, 2);
        // layer 2
        {
            const f4v x0 = *reinterpret_cast<const f4v*>(h1 + 4 * l);
            const f4v x1 = *reinterpret_cast<const f4v*>(h1 + 64 + 4 * l);
            float d[NP2];
#pragma unroll
            for (int p = 0; p < NP2; ++p) {
                float t = 0.0f;
#pragma unroll
                for (int e = 0; e < 4; ++e) t = __builtin_fmaf(x0[e], w2r[p][0][e], t);
#pragma unroll
                for (int e = 0; e < 4; ++e) t = __builtin_fmaf(x1[e], w2r[p][1][e], t);
                d[p] = t;
            }
#pragma unroll
            for (int p = 0; p < NP2; ++p) d[p] = sq_sum16(d[p]);
            float mine = d[0];
#pragma unroll
            for (int p = 1; p < NP2; ++p) mine = l == p ? d[p] : mine;
            if (l < NP2 && o2 < H) h2[o2] = tanhf(mine + bias2);
        }
        __syncthreads();
        if (m == 0) sq_stamp(a, i, 3);
        // layer 3
        {
            const f4v x0 = *reinterpret_cast<const f4v*>(h2 + 4 * l);
            const f4v x1 = *reinterpret_cast<const f4v*>(h2 + 64 + 4 * l);
            float d[NP3];
#pragma unroll
            for (int p = 0; p < NP3; ++p) {
                float t = 0.0f;
#pragma unroll
                for (int e = 0; e < 4; ++e) t = __builtin_fmaf(x0[e], w3r[p][0][e], t);
#pragma unroll
                for (int e = 0; e < 4; ++e) t = __builtin_fmaf(x1[e], w3r[p][1][e], t);
                d[p] = t;
            }
#pragma unroll
            for (int p = 0; p < NP3; ++p) d[p] = sq_sum16(d[p]);
            float mine = d[0];
#pragma unroll
            for (int p = 1; p < NP3; ++p) mine = l == p ? d[p] : mine;
            if (l < NP3 && o2 < P) lg[o2] = mine + bias3;
        }
        (void)HA;
    }
    __syncthreads();
    if (tid >= 64) return;
    if (m == 0) sq_stamp(a, i, 4);
    float out, lad;
    bool in, nd;
    sq_spline_inv<K>(lg, zv, a.c, out, lad, in, nd);
    if (tid != 0) return;
    if (m == 0) sq_stamp(a, i, 5);
    a.x[(int64_t)m * a.ldx + i] = out;
    const float acc = ldprev + lad;
    if (i + 1 < a.dim) {
        a.ldacc[m] = acc;
        const float arg = (a.pi * out) / a.bnd;  // (pi x) / B, flows.py:173's operation order
        float sv, cv;
        sincosf(arg, &sv, &cv);
        a.feat[(int64_t)m * a.dim + i] = cv;
        a.feat[((int64_t)a.M + m) * a.dim + i] = sv;
    } else if (a.logdet != nullptr && a.mode != 0) {
        a.logdet[m] = a.mode == 2 ? a.logdet[m] + acc : acc;
    }
    if (a.status != nullptr) {
        const int bits = (in ? NFK_ST_INSIDE_SEEN : 0) | (in && nd ? NFK_ST_NEG_DISC : 0);
        if (bits != 0) atomicOr(a.status + i, bits);  // (no read first: one round trip less)
    }
    if (m == 0) sq_stamp(a, i, 6);
}

// one launch per column i: workgroups 0 .. M-1 finish conditioner i (one row
// each); workgroups M .. M + 2 nch_next - 1 run the layer-1 chunks of
// conditioner i + 1 that do not need x_i (two per 64 features: the halves of
// its units; double-buffered partial sums by parity); the last 8 read the
// operands of conditioner i + 1's finish into every XCD's L2
template <int K>
// (the conditioners' tensor pointers are kernel arguments: read from a device
// table they were one more dependent memory round trip per launch)
__global__ __launch_bounds__(kSqThreads, 1) void k_sq_step(SqArgs a, SqCond cur, SqCond next, int i, int nch,
                                                           int nch_next) {
    extern __shared__ float sq_smem[];
    const int b = blockIdx.x;
    if (b < a.M)
        sq_finish<K>(a, cur, i, nch, b, sq_smem);
    else if (b < a.M + 2 * nch_next)
        sq_l1_chunk(a, next.W1, i + 1, b - a.M, sq_smem);
    else
        sq_prefetch(a, next, i + 1, 3 * K - 1);
}

int sq_status() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        nfk_set_error("nfk_ar_seqinv: launch failed");
        return (int)e;
    }
    return 0;
}

int sq_chunks(int dim) { return (int)((2LL * (dim - 1) + kSqFC - 1) / kSqFC); }

unsigned long long* g_sq_tdbg = nullptr;

// NFK_SQ_PREFETCH=0 drops the prefetch workgroups (A/B)
bool sq_prefetch_on() {
    static const bool on = [] {
        const char* e = std::getenv("NFK_SQ_PREFETCH");
        return !(e != nullptr && e[0] == '0');
    }();
    return on;
}

}  // namespace

// diagnostic: a device buffer of dim * 12 uint64 for the phase clocks of the
// next nfk_ar_seqinv calls (null: off).  Returns the previous buffer.
extern "C" void* nfk_debug_sq_timing(void* buf) {
    void* prev = g_sq_tdbg;
    g_sq_tdbg = static_cast<unsigned long long*>(buf);
    return prev;
}

extern "C" int nfk_ar_seqinv_supported(int32_t dim, int32_t hidden, int32_t K) {
    const bool k_ok = K == 4 || K == 8 || K == 10 || K == 16 || K == 32;
    // (k_sq_step's LDS: the row's layer-1 chunks, the activations, one weight matrix)
    const bool lds_ok = dim >= 2 && sq_lds(sq_chunks(dim), hidden, K) <= (size_t)160 * 1024;
    static_assert(kSqMaxH <= kSqThreads && 3 * 32 - 1 <= kSqThreads, "sq_finish: one unit / logit per thread");
    // (hidden >= 4: the layer halves' split point KS stays inside a row)
    return (dim >= 2 && dim <= 65536 && hidden >= 4 && hidden <= kSqMaxH && k_ok && lds_ok) ? 1 : 0;
}

extern "C" int64_t nfk_ar_seqinv_workspace(int32_t dim, int32_t hidden, int32_t K, int64_t batch) {
    if (!nfk_ar_seqinv_supported(dim, hidden, K) || batch <= 0) return 0;
    const int64_t M = batch < kSqMaxRows ? batch : kSqMaxRows;
    return 2 * M * dim + 2LL * sq_chunks(dim) * M * hidden + M + kSqThreads;
}

extern "C" int nfk_ar_seqinv(const float* z, int64_t ldz, const float* const* weights, const float* init_param,
                             int32_t dim, int32_t hidden, int32_t K, double tail_bound, float* x, int64_t ldx,
                             float* logdet, int32_t logdet_mode, int64_t batch, int32_t* status, float* workspace,
                             int64_t workspace_floats, nfk_stream_t stream) {
    if (!nfk_ar_seqinv_supported(dim, hidden, K)) return nfk_set_error("nfk_ar_seqinv: shape not supported");
    if (batch < 0) return nfk_set_error("nfk_ar_seqinv: bad batch");
    if (batch == 0) return 0;
    if (!z || !weights || !init_param || !x || !workspace) return nfk_set_error("nfk_ar_seqinv: null pointer");
    if (logdet_mode != 0 && !logdet) return nfk_set_error("nfk_ar_seqinv: null logdet");
    if (ldz < dim || ldx < dim) return nfk_set_error("nfk_ar_seqinv: bad leading dimension");
    if (workspace_floats < nfk_ar_seqinv_workspace(dim, hidden, K, batch))
        return nfk_set_error("nfk_ar_seqinv: workspace too small (nfk_ar_seqinv_workspace)");
    hipStream_t st = (hipStream_t)stream;
    // (a HOST table: each launch takes its conditioners' pointers as arguments)
    auto cond = [&](int j) {  // conditioner j = 1 .. dim-1 (j out of range: conditioner 1, unused)
        const float* const* w = weights + 6 * ((j >= 1 && j < dim ? j : 1) - 1);
        return SqCond{w[0], w[1], w[2], w[3], w[4], w[5]};
    };
    for (int64_t r0 = 0; r0 < batch; r0 += kSqMaxRows) {
        const int M = (int)(batch - r0 < kSqMaxRows ? batch - r0 : kSqMaxRows);
        SqArgs a;
        a.init = init_param;
        a.z = z + r0 * ldz;
        a.ldz = ldz;
        a.x = x + r0 * ldx;
        a.ldx = ldx;
        a.feat = workspace;
        a.part = workspace + 2LL * M * dim;
        a.ldacc = a.part + 2LL * sq_chunks(dim) * M * hidden;
        a.nchmax = sq_chunks(dim);
        a.sink = a.ldacc + M;
        a.logdet = logdet_mode != 0 ? logdet + r0 : nullptr;
        a.status = status;
        a.mode = logdet_mode;
        a.dim = dim;
        a.H = hidden;
        a.M = M;
        a.pi = (float)M_PI;  // torch.tensor(np.pi) times an fp32 tensor: an fp32 product
        a.bnd = (float)tail_bound;
        // unconstrained_RQS(..., tail_bound=B) with the default minimum bin sizes (flows.py:206-207)
        a.c = nfk_make_const(K, -tail_bound, tail_bound, -tail_bound, tail_bound, 1, 1e-3, 1e-3, 1e-3);
        a.tdbg = g_sq_tdbg;
        static bool attr = false;
        if (!attr) {
#define NFK_SQ_ATTR(k)                                                                                         \
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sq_step<k>), hipFuncAttributeMaxDynamicSharedMemorySize, \
                              160 * 1024);
            NFK_SQ_ATTR(4) NFK_SQ_ATTR(8) NFK_SQ_ATTR(10) NFK_SQ_ATTR(16) NFK_SQ_ATTR(32)
#undef NFK_SQ_ATTR
            attr = true;
        }
        // column 0's launch also runs conditioner 1's chunks (none: its two
        // features are x_0's); column i's, conditioner i + 1's
        for (int i = 0; i < dim; ++i) {
            const int nch = (2 * i + kSqFC - 1) / kSqFC;
            const int nxt = i + 1 < dim ? (2 * (i + 1) + kSqFC - 1) / kSqFC : 0;
            const int pre = i + 1 < dim && sq_prefetch_on() ? 8 : 0;  // (one prefetch workgroup per XCD)
            const SqCond cur = cond(i), next = cond(i + 1);
            const size_t lds = sq_lds(nch, hidden, K);
#define NFK_SQ_STEP(k) \
    if (K == k)    \
        hipLaunchKernelGGL(k_sq_step<k>, dim3((unsigned)(M + 2 * nxt + pre)), dim3(kSqThreads), lds, st, a, cur, next, \
                           i, nch, nxt);
            NFK_SQ_STEP(4) NFK_SQ_STEP(8) NFK_SQ_STEP(10) NFK_SQ_STEP(16) NFK_SQ_STEP(32)
#undef NFK_SQ_STEP
            if (int e = sq_status()) return e;
        }
    }
    return 0;
}
