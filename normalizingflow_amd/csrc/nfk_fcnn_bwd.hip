// nfk_fcnn_bwd.hip -- input-gradient GEMMs of the FCNN conditioner's
// backward (nf/flows.py:20-35 differentiated; normalizingflow_amd/fcnn_grad.py)
// on the matrix cores, with tanh's backward fused into the epilogue:
//
//   out[b, j] = (sum_p g[b, p] W[p, j]) * (1 - h[b, j]^2)     (h nullable: no tanh factor)
//
// g [B, P] is the gradient reaching a Linear's output, W [P, H] its nn.Linear
// weight (out x in), h [B, H] the tanh activation feeding that Linear.  At
// c3 that is dL/dh2 = gp W3 (P = 736, H = 100; then x (1 - h2^2)), the next
// Linear's 100 x 100, and the last one's 100 x 32 without tanh.
//
// Arithmetic: the fp16 two-way split of the fused forward (hi*hi + hi*lo +
// lo*hi on v_mfma_f32_16x16x32_f16, fp32 accumulation).  g is scaled per row
// by a power of two that puts the row's max |g| (so far) just under 2^14 (every
// output column is one row, so the scale comes off exactly in the epilogue); W by one
// power of two for the whole matrix (nfk_fcnn_dh_pack).
//
// Layout: a wave owns 16 rows of g (b) and every output feature (NT tiles of
// 16 j); the transposed weight streams through two LDS slots one 32-wide
// k-step at a time (NT tiles x {hi, lo} x 1 KiB), shared by the 8 waves of a
// workgroup.  g is read once, under a running per-row scale (see k_dh): HBM
// sees g once, h once and out once.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../../include/nfk.h"

int nfk_set_error(const char* msg);

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kDhWaves = 8;
constexpr int kDhMaxNT = 8;  // H <= 128

int launch_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        char buf[200];
        std::snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
        nfk_set_error(buf);
        return (int)e;
    }
    return 0;
}

__device__ __forceinline__ f32x4 mfma16(h8 a, h8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// pack: [0] = 1 / weight scale, then from half offset 128 the fragments
// [kb][t][part][lane][e] = part of W[p = 32 kb + 8 (lane >> 4) + e][j = 16 t + (lane & 15)] * s
// (part 0 = hi, 1 = lo; zero outside P x H).  Two launches: max |W| (a
// grid-stride pass whose waves atomicMax the bit pattern into pack[2], zeroed
// first: non-negative floats order as integers, so the result is exact and
// order-independent), then the words; pack[0] = 1 / s is written by thread 0.
__global__ __launch_bounds__(256) void k_dh_scale(const float* __restrict__ W, int n, float* pack) {
    float mx = 0.0f;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        mx = fmaxf(mx, fabsf(W[i]));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
    if ((threadIdx.x & 63) == 0 && mx > 0.0f)
        atomicMax(reinterpret_cast<int*>(pack) + 2, __float_as_int(fminf(mx, 3.0e38f)));
}

__global__ __launch_bounds__(256) void k_dh_pack(const float* __restrict__ W, int P, int H, int KB, int NT,
                                                 float* pack) {
    const float mx = __int_as_float(reinterpret_cast<const int*>(pack)[2]);
    int ex = 0;
    if (mx > 0.0f) frexpf(mx, &ex);
    const float s = ldexpf(1.0f, 14 - ex);
    if (blockIdx.x == 0 && threadIdx.x == 0) pack[0] = ldexpf(1.0f, ex - 14);  // 1 / s
    _Float16* body = reinterpret_cast<_Float16*>(pack) + 128;
    const int n = KB * NT * 2 * 64 * 8;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int e = i & 7, lane = (i >> 3) & 63, part = (i >> 9) & 1, t = (i >> 10) % NT, kb = (i >> 10) / NT;
        const int p = 32 * kb + 8 * (lane >> 4) + e, j = 16 * t + (lane & 15);
        const float v = (p < P && j < H) ? W[(int64_t)p * H + j] * s : 0.0f;
        const _Float16 hi = (_Float16)v;
        body[i] = part == 0 ? hi : (_Float16)(v - (float)hi);
    }
}

template <int NT>
__global__ __launch_bounds__(64 * kDhWaves) void k_dh(const float* __restrict__ g, int64_t ldg, int P,
                                                      const float* __restrict__ pack, const float* __restrict__ h,
                                                      int64_t ldh, int H, float* __restrict__ out, int64_t ldo,
                                                      int64_t cso, int acc_out, const float* __restrict__ bias,
                                                      int tanh_out, int64_t B) {
    constexpr int SLOT = NT * 2 * 64;  // h8 fragments per k-step
    __shared__ h8 slot[2][SLOT];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, q = lane >> 4, n = lane & 15;
    const int KB = (P + 31) / 32;
    const int64_t row = ((int64_t)blockIdx.x * kDhWaves + wid) * 16 + n;
    const bool rok = row < B;
    const float* gr = g + (rok ? row : B - 1) * ldg;
    const h8* body = reinterpret_cast<const h8*>(reinterpret_cast<const _Float16*>(pack) + 128);

    // g is split under a running per-row scale: 2^(14 - ex) with ex the
    // exponent of the largest |g| of the row seen so far (the row's 4 lanes
    // agree through two shuffles).  When a k-step raises ex, the row's
    // accumulators (all in this lane: every D element of a lane is sample n)
    // are rescaled by the exact power of two.  One pass over g, prefetched a
    // k-step ahead.
    auto load = [&](int kb, float4& u, float4& v) {
        const int p0 = 32 * kb + 8 * q;
        u = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        v = u;
        if (p0 < P) u = *reinterpret_cast<const float4*>(gr + p0);
        if (p0 + 4 < P) v = *reinterpret_cast<const float4*>(gr + p0 + 4);
    };

    // k-step 0 into slot 0
    for (int i = threadIdx.x; i < SLOT; i += 64 * kDhWaves) slot[0][i] = body[i];
    // g two k-steps ahead: (u, v) this step, (u1, v1) the next
    float4 u, v, u1, v1;
    load(0, u, v);
    if (KB > 1) load(1, u1, v1);
    __syncthreads();

    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    int es = 100;  // running scale exponent: g is split as g 2^es, 2^es max|g| so far < 2^14
    constexpr int PER = (SLOT + 64 * kDhWaves - 1) / (64 * kDhWaves);
    for (int kb = 0; kb < KB; ++kb) {
        const int cur = kb & 1;
        // the next k-step: weight fragments and g into registers
        h8 nx[PER];
        float4 un, vn;
        if (kb + 1 < KB) {
#pragma unroll
            for (int r = 0; r < PER; ++r) {
                const int i = threadIdx.x + r * 64 * kDhWaves;
                if (i < SLOT) nx[r] = body[(int64_t)(kb + 1) * SLOT + i];
            }
        }
        if (kb + 2 < KB) load(kb + 2, un, vn);
        float mx = fmaxf(fmaxf(fmaxf(fabsf(u.x), fabsf(u.y)), fmaxf(fabsf(u.z), fabsf(u.w))),
                         fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        int e2 = es;
        if (mx > 0.0f && mx < 3.0e38f) {
            int em = 0;
            frexpf(mx, &em);  // mx < 2^em
            e2 = (14 - em) < es ? (14 - em) : es;
        }
        if (e2 != es) {
            const float r = ldexpf(1.0f, e2 - es);
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = acc[t] * r;
            es = e2;
        }
        const float sg = ldexpf(1.0f, es);
        const float xv[8] = {u.x * sg, u.y * sg, u.z * sg, u.w * sg, v.x * sg, v.y * sg, v.z * sg, v.w * sg};
        h8 bh, bl;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const _Float16 hh = (_Float16)xv[e];
            bh[e] = hh;
            bl[e] = (_Float16)(xv[e] - (float)hh);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const h8 ahi = slot[cur][(2 * t) * 64 + lane], alo = slot[cur][(2 * t + 1) * 64 + lane];
            acc[t] = mfma16(alo, bh, acc[t]);
            acc[t] = mfma16(ahi, bl, acc[t]);
            acc[t] = mfma16(ahi, bh, acc[t]);
        }
        if (kb + 1 < KB) {
#pragma unroll
            for (int r = 0; r < PER; ++r) {
                const int i = threadIdx.x + r * 64 * kDhWaves;
                if (i < SLOT) slot[cur ^ 1][i] = nx[r];
            }
        }
        u = u1;
        v = v1;
        if (kb + 2 < KB) {
            u1 = un;
            v1 = vn;
        }
        __syncthreads();
    }

    if (!rok) return;
    const float inv = ldexpf(1.0f, -es) * pack[0];
    // 4 consecutive features j0 .. j0 + 3 of one row per tile: one 16-byte h
    // load and out store where the rows allow it
    const bool vec = cso == 1 && ((ldh & 3) == 0 || h == nullptr) && (ldo & 3) == 0 &&
                     ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(h)) & 15) == 0;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int j0 = 16 * t + 4 * q;
        if (j0 >= H) continue;
        float d[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            // forward form (nfk_fcnn_linear): + bias, then tanh
            d[r] = acc[t][r] * inv;
            if (bias != nullptr && j0 + r < H) d[r] += bias[j0 + r];
            if (tanh_out) d[r] = tanhf(d[r]);
        }
        if (vec && j0 + 4 <= H) {
            if (h != nullptr) {
                const float4 hv = *reinterpret_cast<const float4*>(h + row * ldh + j0);
                d[0] *= 1.0f - hv.x * hv.x;
                d[1] *= 1.0f - hv.y * hv.y;
                d[2] *= 1.0f - hv.z * hv.z;
                d[3] *= 1.0f - hv.w * hv.w;
            }
            float4* o = reinterpret_cast<float4*>(out + row * ldo + j0);
            if (acc_out) {
                const float4 w = *o;
                d[0] += w.x;
                d[1] += w.y;
                d[2] += w.z;
                d[3] += w.w;
            }
            *o = make_float4(d[0], d[1], d[2], d[3]);
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int j = j0 + r;
                if (j < H) {
                    float v = d[r];
                    if (h != nullptr) {
                        const float hv = h[row * ldh + j];
                        v *= 1.0f - hv * hv;
                    }
                    float* o = out + row * ldo + (int64_t)j * cso;
                    *o = acc_out ? *o + v : v;
                }
            }
        }
    }
}

}  // namespace

namespace {
// out[b, j] = x[b, cols[j]] (j < n), out[b, n] = 1, out[b, n + 1 .. ldo) = 0:
// one thread per float4 of an output row, the gathers of a wave spread over
// a few consecutive x rows (their cache lines read once)
__global__ __launch_bounds__(256) void k_gather_cols1(const float* __restrict__ x, int64_t ldx,
                                                      const int32_t* __restrict__ cols, int n, int64_t batch,
                                                      float* __restrict__ out, int64_t ldo) {
    const int q4 = (int)(ldo >> 2);
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t r = t / q4;
    if (r >= batch) return;
    const int j0 = 4 * (int)(t - r * q4);
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int j = j0 + k;
        v[k] = j < n ? x[r * ldx + cols[j]] : (j == n ? 1.0f : 0.0f);
    }
    *reinterpret_cast<float4*>(out + r * ldo + j0) = make_float4(v[0], v[1], v[2], v[3]);
}
}  // namespace

extern "C" int nfk_gather_cols_ones(const float* x, int64_t ldx, const int32_t* cols, int32_t n, int64_t batch,
                                    float* out, int64_t ldo, nfk_stream_t stream) {
    if (n < 0 || batch < 0 || ldo < n + 1 || (ldo & 3)) return nfk_set_error("nfk_gather_cols_ones: bad shape");
    if (batch == 0) return 0;
    if (!x || !out || (n > 0 && !cols)) return nfk_set_error("nfk_gather_cols_ones: null pointer");
    if (reinterpret_cast<uintptr_t>(out) & 15) return nfk_set_error("nfk_gather_cols_ones: out must be 16-byte aligned");
    const int64_t threads = batch * (ldo >> 2);
    hipLaunchKernelGGL(k_gather_cols1, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x,
                       ldx, cols, n, batch, out, ldo);
    return launch_status("nfk_gather_cols_ones");
}

extern "C" int64_t nfk_fcnn_dh_pack_floats(int32_t P, int32_t H) {
    if (P <= 0 || H <= 0 || H > 16 * kDhMaxNT || (P & 3)) return 0;
    const int64_t KB = (P + 31) / 32, NT = (H + 15) / 16;
    return 64 + KB * NT * 2 * 64 * 8 / 2;
}

extern "C" int nfk_fcnn_dh_pack(const float* W, int32_t P, int32_t H, float* pack, nfk_stream_t stream) {
    if (nfk_fcnn_dh_pack_floats(P, H) == 0) return nfk_set_error("nfk_fcnn_dh_pack: unsupported shape");
    if (!W || !pack) return nfk_set_error("nfk_fcnn_dh_pack: null pointer");
    hipStream_t st = (hipStream_t)stream;
    const int KB = (P + 31) / 32, NT = (H + 15) / 16;
    const int n = KB * NT * 2 * 64 * 8;
    if (hipMemsetAsync(pack, 0, 4 * sizeof(float), st) != hipSuccess)
        return nfk_set_error("nfk_fcnn_dh_pack: memset failed");
    const int sb = (P * H + 4095) / 4096;
    hipLaunchKernelGGL(k_dh_scale, dim3((unsigned)(sb < 256 ? sb : 256)), dim3(256), 0, st, W, P * H, pack);
    hipLaunchKernelGGL(k_dh_pack, dim3((unsigned)((n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024)), dim3(256), 0,
                       st, W, P, H, KB, NT, pack);
    return launch_status("nfk_fcnn_dh_pack");
}

namespace {
int dh_launch(const float* g, int64_t ldg, int32_t P, const float* pack, const float* h, int64_t ldh, int32_t H,
              float* out, int64_t ldo, int64_t out_col_stride, int32_t accumulate, const float* bias, int tanh_out,
              int64_t batch, hipStream_t st);
}

extern "C" int nfk_fcnn_dh(const float* g, int64_t ldg, int32_t P, const float* pack, const float* h, int64_t ldh,
                           int32_t H, float* out, int64_t ldo, int64_t out_col_stride, int32_t accumulate,
                           int64_t batch, nfk_stream_t stream) {
    return dh_launch(g, ldg, P, pack, h, ldh, H, out, ldo, out_col_stride, accumulate, nullptr, 0, batch,
                     (hipStream_t)stream);
}

extern "C" int nfk_fcnn_linear(const float* x, int64_t ldx, int32_t P, const float* pack, const float* bias,
                               int32_t tanh_out, int32_t H, float* out, int64_t ldo, int64_t batch,
                               nfk_stream_t stream) {
    return dh_launch(x, ldx, P, pack, nullptr, 0, H, out, ldo, 1, 0, bias, tanh_out ? 1 : 0, batch,
                     (hipStream_t)stream);
}

namespace {
int dh_launch(const float* g, int64_t ldg, int32_t P, const float* pack, const float* h, int64_t ldh, int32_t H,
              float* out, int64_t ldo, int64_t out_col_stride, int32_t accumulate, const float* bias, int tanh_out,
              int64_t batch, hipStream_t st) {
    if (out_col_stride < 1) return nfk_set_error("nfk_fcnn_dh: bad output column stride");
    if (nfk_fcnn_dh_pack_floats(P, H) == 0 || batch < 0) return nfk_set_error("nfk_fcnn_dh: unsupported shape");
    if (batch == 0) return 0;
    if (!g || !pack || !out) return nfk_set_error("nfk_fcnn_dh: null pointer");
    if ((ldg & 3) || (reinterpret_cast<uintptr_t>(g) & 15))
        return nfk_set_error("nfk_fcnn_dh: g rows must be 16-byte aligned");
    const int64_t blocks = (batch + 16 * kDhWaves - 1) / (16 * kDhWaves);
    const int NT = (H + 15) / 16;
#define CASE(nt)                                                                                                   \
    case nt:                                                                                                       \
        hipLaunchKernelGGL(k_dh<nt>, dim3((unsigned)blocks), dim3(64 * kDhWaves), 0, st, g, ldg, P, pack, h, ldh, H, \
                           out, ldo, out_col_stride, accumulate ? 1 : 0, bias, tanh_out, batch);                   \
        break;
    switch (NT) {
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
        default: return nfk_set_error("nfk_fcnn_dh: H too large");
    }
#undef CASE
    return launch_status("nfk_fcnn_dh");
}
}  // namespace
