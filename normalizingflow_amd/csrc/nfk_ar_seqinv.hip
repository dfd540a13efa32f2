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
//                           layer (95 logits), the spline's inverse
//                           (nfk_rqs_element_lean: the reference's 2B softmax /
//                           softplus, then RQS, utils.py:27-152), x[m, i], the
//                           row's log|det| in column order (flows.py:208), the
//                           status word of column i, cos / sin (pi x_i / B)
//   workgroups M ..         layer 1 of conditioner i + 1 over its features in
//                           64-feature chunks, all but x_i's two (which the
//                           first group is computing): [M, 64] x [64, H]
//                           register tiles, fp32 partial sums (double-buffered
//                           by conditioner parity)
//
// The conditioners' nn.Linear weights are read in place (fp32, a device table
// of their pointers: the fused pack's table), and the arithmetic is fp32 FMA
// throughout: the inverse is latency-bound (4,095 dependent launches per layer
// at Polymer's shape), not bandwidth- or FLOP-bound, and every weight is read
// once per layer (1.68 GB at Polymer, 0.2 ms of HBM time).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../include/nfk.h"
#include "nfk_spline.h"

int nfk_set_error(const char* msg);  // nfk_kernels.hip
NfkSplineConst nfk_make_const(int K, double left, double right, double bottom, double top, int tails, double min_w,
                              double min_h, double min_d);

namespace {

constexpr int kSqFC = 64;        // layer-1 features per chunk workgroup
constexpr int kSqThreads = 256;  // both kernels
constexpr int kSqMaxRows = 64;   // rows per pass
constexpr int kSqMaxH = 128;     // hidden width (the chunks' 4 x 4 register tiles: 64 rows x 128)

struct SqArgs {
    const float* const* w;  // [6 (dim - 1)]: conditioner i = 1 .. dim-1: W1 [H, 2i], b1, W2 [H, H], b2, W3 [P, H], b3
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
};

// diagnostic: thread 0 of row 0's finish and of the first chunk workgroup stamp
// the shader clock at their phase boundaries, [dim][12] per pass
__device__ __forceinline__ void sq_stamp(const SqArgs& a, int i, int slot) {
    if (a.tdbg != nullptr && threadIdx.x == 0) a.tdbg[(int64_t)i * 12 + slot] = __builtin_readcyclecounter();
}

// LDS of a k_sq_step workgroup: the finish part's (the row's layer-1 chunks,
// h1, h2, logits, one weight matrix at a time) or the layer-1 part's
// (64 features x 128 units of weights, 64 features x 64 rows), the larger
inline size_t sq_fin_floats(int nch, int H, int K) {
    const int P = 3 * K - 1;
    auto al = [](int64_t v) { return (v + 3) & ~3LL; };
    const int S = H | 1;  // (the staged W2 / W3 rows' stride, sq_finish)
    return (size_t)(al((int64_t)nch * H) + 2 * al(H) + al(P) + al((int64_t)H * S) + al((int64_t)P * S));
}
inline size_t sq_lds(int nch, int H, int K) {
    const size_t l1 = (size_t)kSqFC * (kSqMaxH + kSqMaxRows);
    const size_t f = sq_fin_floats(nch, H, K);
    return (f > l1 ? f : l1) * sizeof(float);
}

// LDS <- global with U loads in flight per thread (one load, one wait, one
// store per element made every staging loop a chain of HBM round trips:
// 38.8 us per column at Polymer's shape)
template <int U>
__device__ __forceinline__ void sq_stage(float* __restrict__ dst, const float* __restrict__ src, int n) {
    for (int b = threadIdx.x; b < n; b += kSqThreads * U) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = b + u * kSqThreads;
            v[u] = e < n ? src[e] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = b + u * kSqThreads;
            if (e < n) dst[e] = v[u];
        }
    }
}

// the same with 16-byte loads where both ends are 16-byte aligned and n % 4 == 0
template <int U>
__device__ __forceinline__ void sq_stage4(float* __restrict__ dst, const float* __restrict__ src, int n) {
    if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) != 0 || (n & 3) != 0) {
        sq_stage<U>(dst, src, n);
        return;
    }
    const int n4 = n >> 2;
    const float4* s4 = reinterpret_cast<const float4*>(src);
    float4* d4 = reinterpret_cast<float4*>(dst);
    for (int b = threadIdx.x; b < n4; b += kSqThreads * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = b + u * kSqThreads;
            if (e < n4) v[u] = s4[e];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = b + u * kSqThreads;
            if (e < n4) d4[e] = v[u];
        }
    }
}

typedef float sq_f4 __attribute__((ext_vector_type(4)));  // (HIP's float4 struct arrays went to scratch)

// row r, column c of a row-major [., H] matrix from its flat index (a float
// estimate, then corrected: exact for the staged sizes)
__device__ __forceinline__ void sq_rc(int flat, int H, float invH, int& r, int& c) {
    r = (int)((float)flat * invH);
    c = flat - r * H;
    if (c >= H) {
        ++r;
        c -= H;
    } else if (c < 0) {
        --r;
        c += H;
    }
}

// four consecutive elements (flat index flat0) of a row-major [., H] matrix
// into LDS rows of stride S = H | 1: an odd stride, so the layer dots (lane h
// reading row h) hit 64 different banks.  H >= 4: at most one row break.
__device__ __forceinline__ void sq_put4(float* dst, int flat0, sq_f4 v, int H, int S, float invH) {
    int r, c;
    sq_rc(flat0, H, invH, r, c);
    const int base = r * S + c, d = S - H;
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[base + q + (c + q >= H ? d : 0)] = v[q];
}

// the same staging, element by element, for elements from .. n - 1
template <int U>
__device__ __forceinline__ void sq_stage_pad(float* __restrict__ dst, const float* __restrict__ src, int from, int n,
                                             int H, int S, float invH) {
    for (int b = from + threadIdx.x; b < n; b += kSqThreads * U) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = b + u * kSqThreads;
            v[u] = e < n ? src[e] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = b + u * kSqThreads;
            if (e < n) {
                int r, c;
                sq_rc(e, H, invH, r, c);
                dst[r * S + c] = v[u];
            }
        }
    }
}

// layer 1 of conditioner j over features f0 .. f0 + 63 (chunk c), WITHOUT the
// two features of coordinate j - 1 (cos at f = j - 1, sin at f = 2j - 1: the
// finish of column j - 1 runs in the same launch and writes them; the finish of
// conditioner j adds their products itself).  The chunk's weights and the rows'
// features through LDS ([f][h], [f][m]); each thread a 4-row x 4-unit tile
__device__ void sq_l1_chunk(const SqArgs& a, int j, int c, float* lds) {
    float(*ws)[kSqMaxH] = reinterpret_cast<float(*)[kSqMaxH]>(lds);
    float(*fs)[kSqMaxRows] = reinterpret_cast<float(*)[kSqMaxRows]>(lds + kSqFC * kSqMaxH);
    const int F = 2 * j, f0 = c * kSqFC, nf = F - f0 < kSqFC ? F - f0 : kSqFC;
    const int H = a.H, M = a.M;
    if (c == 0) sq_stamp(a, j - 1, 8);
    const float* W1 = a.w[6 * (j - 1)];
    // (feature pairs: F = 2j is even, so every row segment is 8-byte aligned;
    // 16 loads in flight per thread, consecutive threads along one weight row)
    constexpr int FC2 = kSqFC / 2;
    const float2* W1p = reinterpret_cast<const float2*>(W1);
    for (int b = threadIdx.x; b < H * FC2; b += kSqThreads * 16) {
        float2 v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int e = b + u * kSqThreads, h = e / FC2, f = 2 * (e - h * FC2);
            v[u] = (e < H * FC2 && f < nf) ? W1p[((int64_t)h * F + f0 + f) >> 1] : make_float2(0.0f, 0.0f);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int e = b + u * kSqThreads, h = e / FC2, f = 2 * (e - h * FC2);
            if (e < H * FC2) {
                ws[f][h] = v[u].x;
                ws[f + 1][h] = v[u].y;
            }
        }
    }
    // feature f of conditioner j: cos(pi x_f / B) for f < j, sin(pi x_(f-j) / B)
    // above (trig_transform's cat, flows.py:172-173)
    for (int b = threadIdx.x; b < M * kSqFC; b += kSqThreads * 16) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int e = b + u * kSqThreads, m = e / kSqFC, f = e - m * kSqFC, g = f0 + f;
            v[u] = 0.0f;
            if (e < M * kSqFC && f < nf && g != j - 1 && g != 2 * j - 1)
                v[u] = g < j ? a.feat[(int64_t)m * a.dim + g] : a.feat[((int64_t)M + m) * a.dim + (g - j)];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int e = b + u * kSqThreads, m = e / kSqFC, f = e - m * kSqFC;
            if (e < M * kSqFC) fs[f][m] = v[u];
        }
    }
    __syncthreads();
    if (c == 0) sq_stamp(a, j - 1, 9);
    float* part = a.part + (int64_t)(j & 1) * M * a.nchmax * H;
    const int HT = (H + 3) / 4, MT4 = (M + 3) / 4;
    for (int t = threadIdx.x; t < HT * MT4; t += kSqThreads) {
        const int h0 = 4 * (t % HT), m0 = 4 * (t / HT);
        float acc[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int u = 0; u < 4; ++u) acc[r][u] = 0.0f;
        for (int f = 0; f < nf; ++f) {
            float fv[4], wv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) fv[r] = fs[f][(m0 + r) & (kSqMaxRows - 1)];
#pragma unroll
            for (int u = 0; u < 4; ++u) wv[u] = ws[f][(h0 + u) & (kSqMaxH - 1)];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int u = 0; u < 4; ++u) acc[r][u] = __builtin_fmaf(fv[r], wv[u], acc[r][u]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (m0 + r < M && h0 + u < H) part[((int64_t)(m0 + r) * a.nchmax + c) * H + h0 + u] = acc[r][u];
    }
    if (c == 0) sq_stamp(a, j - 1, 10);
}

// the rest of conditioner i for ONE row m: its layer-1 chunks summed in order,
// + the products of coordinate i - 1's two features (left out of the chunks),
// + b1, tanh, layer 2, tanh, the output layer, the spline's inverse, x[m, i],
// the row's log|det|, the status word, cos / sin of x[m, i]
template <int K>
__device__ void sq_finish(const SqArgs& a, int i, int nch, int m, float* lds) {
    constexpr int P = 3 * K - 1;
    const int H = a.H, tid = threadIdx.x;
    // (16-byte aligned regions: the staged matrices are copied by float4)
    const int HA = (H + 3) & ~3, PA = (P + 3) & ~3;
    float* pr = lds;            // [nch][H]
    float* h1 = pr + ((nch * H + 3) & ~3);  // [H]
    float* h2 = h1 + HA;        // [H]
    float* lg = h2 + HA;        // [P]
    float* w2 = lg + PA;        // W2 [H][H] (row-major, as nn.Linear; rows S apart)
    const int S = H | 1;        // (odd row stride: sq_put4)
    float* w3 = w2 + ((H * S + 3) & ~3);  // W3 [P][H]
    // every operand a thread needs from memory is requested up front (a load
    // issued after a barrier is one more dependent round trip on the column's
    // critical path): the biases (H <= 128 and P <= 95 < the workgroup, so one
    // unit / logit per thread), thread 0's z[m, i] and the row's log|det| so far
    if (m == 0) sq_stamp(a, i, 0);
    const float* const* wt = a.w + 6 * (i > 0 ? i - 1 : 0);
    float bias1 = 0.0f, bias2 = 0.0f, bias3 = 0.0f, zv = 0.0f, ldprev = 0.0f;
    if (i > 0) {
        if (tid < H) {
            bias1 = wt[1][tid];
            bias2 = wt[3][tid];
        }
        if (tid < P) bias3 = wt[5][tid];
    }
    if (tid == 0) {
        zv = a.z[(int64_t)m * a.ldz + i];
        ldprev = i == 0 ? 0.0f : a.ldacc[m];
    }
    if (i == 0) {
        // coordinate 0: init_param, the same logits for every row (flows.py:196-199)
        for (int p = tid; p < P; p += kSqThreads) lg[p] = a.init[p];
    } else {
        const float *W1 = wt[0], *W2 = wt[2], *W3 = wt[4];
        // ONE round trip for everything the row needs: its layer-1 partials
        // (contiguous), W2, W3, and x_(i-1)'s two weight columns of W1 -- every
        // load issued before any is waited for (a wait per region had made the
        // finish three or four dependent HBM round trips)
        const float* src = a.part + ((int64_t)(i & 1) * a.M + m) * a.nchmax * H;
        const int np = nch * H, n2 = H * H, n3 = P * H;
        const bool v4 = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(W2) |
                          reinterpret_cast<uintptr_t>(W3)) & 15) == 0 && (np & 3) == 0 && (n2 & 3) == 0 &&
                        (n3 & 3) == 0;
        constexpr int UP = 8, U2 = 12, U3 = 12;
        float wa = 0.0f, wb = 0.0f, cp = 0.0f, sp = 0.0f;
        if (tid < H) {
            const float* wr = W1 + (int64_t)tid * 2 * i;
            wa = wr[i - 1];
            wb = wr[2 * i - 1];
        }
        cp = a.feat[(int64_t)m * a.dim + i - 1];
        sp = a.feat[((int64_t)a.M + m) * a.dim + i - 1];
        if (v4) {
            typedef sq_f4 f4v;
            const float invH = 1.0f / (float)H;
            const f4v *sp4 = reinterpret_cast<const f4v*>(src), *s24 = reinterpret_cast<const f4v*>(W2),
                      *s34 = reinterpret_cast<const f4v*>(W3);
            f4v rp[UP], r2[U2], r3[U3];
#pragma unroll
            for (int u = 0; u < UP; ++u) {
                const int e = tid + u * kSqThreads;
                rp[u] = e < np / 4 ? sp4[e] : f4v{0.0f, 0.0f, 0.0f, 0.0f};
            }
#pragma unroll
            for (int u = 0; u < U2; ++u) {
                const int e = tid + u * kSqThreads;
                r2[u] = e < n2 / 4 ? s24[e] : f4v{0.0f, 0.0f, 0.0f, 0.0f};
            }
#pragma unroll
            for (int u = 0; u < U3; ++u) {
                const int e = tid + u * kSqThreads;
                r3[u] = e < n3 / 4 ? s34[e] : f4v{0.0f, 0.0f, 0.0f, 0.0f};
            }
#pragma unroll
            for (int u = 0; u < UP; ++u) {
                const int e = tid + u * kSqThreads;
                if (e < np / 4) reinterpret_cast<f4v*>(pr)[e] = rp[u];
            }
#pragma unroll
            for (int u = 0; u < U2; ++u) {
                const int e = tid + u * kSqThreads;
                if (e < n2 / 4) sq_put4(w2, 4 * e, r2[u], H, S, invH);
            }
#pragma unroll
            for (int u = 0; u < U3; ++u) {
                const int e = tid + u * kSqThreads;
                if (e < n3 / 4) sq_put4(w3, 4 * e, r3[u], H, S, invH);
            }
            // (larger shapes: the rest by the loop)
            if (np / 4 > UP * kSqThreads) sq_stage<8>(pr + 4 * UP * kSqThreads, src + 4 * UP * kSqThreads, np - 4 * UP * kSqThreads);
            if (n2 / 4 > U2 * kSqThreads) sq_stage_pad<8>(w2, W2, 4 * U2 * kSqThreads, n2, H, S, invH);
            if (n3 / 4 > U3 * kSqThreads) sq_stage_pad<8>(w3, W3, 4 * U3 * kSqThreads, n3, H, S, invH);
        } else {
            sq_stage<16>(pr, src, np);
            const float invH = 1.0f / (float)H;
            sq_stage_pad<16>(w2, W2, 0, n2, H, S, invH);
            sq_stage_pad<16>(w3, W3, 0, n3, H, S, invH);
        }
        __syncthreads();
        if (m == 0) sq_stamp(a, i, 1);
        if (tid < H) {
            float s = 0.0f;
            for (int c = 0; c < nch; ++c) s += pr[c * H + tid];
            s = __builtin_fmaf(cp, wa, s);
            s = __builtin_fmaf(sp, wb, s);
            h1[tid] = tanhf(s + bias1);
        }
        __syncthreads();
        if (m == 0) sq_stamp(a, i, 2);
        if (tid < H) {
            const float* wr = w2 + tid * S;
            float s = 0.0f;
            for (int k = 0; k < H; ++k) s = __builtin_fmaf(h1[k], wr[k], s);
            h2[tid] = tanhf(s + bias2);
        }
        __syncthreads();
        if (m == 0) sq_stamp(a, i, 3);
        if (tid < P) {
            const float* wr = w3 + tid * S;
            float s = 0.0f;
            for (int k = 0; k < H; ++k) s = __builtin_fmaf(h2[k], wr[k], s);
            lg[tid] = s + bias3;
        }
    }
    __syncthreads();
    if (tid != 0) return;
    if (m == 0) sq_stamp(a, i, 4);
    float wr[K], hr[K], dr[K - 1 > 0 ? K - 1 : 1];
#pragma unroll
    for (int p = 0; p < K; ++p) wr[p] = lg[p];
#pragma unroll
    for (int p = 0; p < K; ++p) hr[p] = lg[K + p];
#pragma unroll
    for (int p = 0; p < K - 1; ++p) dr[p] = lg[2 * K + p];
    float out, lad;
    bool in, nd;
    nfk_rqs_element_lean<K, true>(zv, wr, hr, dr, a.c, out, lad, in, nd);
    if (m == 0) sq_stamp(a, i, 5);
    a.x[(int64_t)m * a.ldx + i] = out;
    const float acc = ldprev + lad;
    if (i + 1 < a.dim) {
        a.ldacc[m] = acc;
        const float arg = (a.pi * out) / a.bnd;  // (pi x) / B, flows.py:173's operation order
        a.feat[(int64_t)m * a.dim + i] = cosf(arg);
        a.feat[((int64_t)a.M + m) * a.dim + i] = sinf(arg);
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
// each); workgroups M .. M + nch_next - 1 run the layer-1 chunks of conditioner
// i + 1 that do not need x_i (double-buffered partial sums by parity)
template <int K>
__global__ __launch_bounds__(kSqThreads, 1) void k_sq_step(SqArgs a, int i, int nch, int nch_next) {
    extern __shared__ float sq_smem[];
    const int b = blockIdx.x;
    if (b < a.M)
        sq_finish<K>(a, i, nch, b, sq_smem);
    else
        sq_l1_chunk(a, i + 1, b - a.M, sq_smem);
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
    // (hidden >= 4: sq_put4's single row break)
    return (dim >= 2 && dim <= 65536 && hidden >= 4 && hidden <= kSqMaxH && k_ok && lds_ok) ? 1 : 0;
}

extern "C" int64_t nfk_ar_seqinv_workspace(int32_t dim, int32_t hidden, int32_t K, int64_t batch) {
    if (!nfk_ar_seqinv_supported(dim, hidden, K) || batch <= 0) return 0;
    const int64_t M = batch < kSqMaxRows ? batch : kSqMaxRows;
    return 2 * M * dim + 2LL * sq_chunks(dim) * M * hidden + M;
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
    for (int64_t r0 = 0; r0 < batch; r0 += kSqMaxRows) {
        const int M = (int)(batch - r0 < kSqMaxRows ? batch - r0 : kSqMaxRows);
        SqArgs a;
        a.w = weights;
        a.init = init_param;
        a.z = z + r0 * ldz;
        a.ldz = ldz;
        a.x = x + r0 * ldx;
        a.ldx = ldx;
        a.feat = workspace;
        a.part = workspace + 2LL * M * dim;
        a.ldacc = a.part + 2LL * sq_chunks(dim) * M * hidden;
        a.nchmax = sq_chunks(dim);
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
            const size_t lds = sq_lds(nch, hidden, K);
#define NFK_SQ_STEP(k) \
    if (K == k) hipLaunchKernelGGL(k_sq_step<k>, dim3((unsigned)(M + nxt)), dim3(kSqThreads), lds, st, a, i, nch, nxt);
            NFK_SQ_STEP(4) NFK_SQ_STEP(8) NFK_SQ_STEP(10) NFK_SQ_STEP(16) NFK_SQ_STEP(32)
#undef NFK_SQ_STEP
            if (int e = sq_status()) return e;
        }
    }
    return 0;
}
