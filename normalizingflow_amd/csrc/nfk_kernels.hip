// nfk_kernels.hip -- streaming (HBM-bound) kernels of the coupling-layer hot
// path for MI355X / gfx950, and their C-ABI entry points (include/nfk.h).
//
// Built with -ffp-contract=off so every fp32 op rounds separately, as the
// reference's chain of ATen ops does.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>

#include "../../include/nfk.h"
#include "nfk_spline.h"

// ---------------------------------------------------------------------------
// error plumbing
// ---------------------------------------------------------------------------
static thread_local char g_err[256] = "";

int nfk_set_error(const char* msg) {
    std::snprintf(g_err, sizeof(g_err), "%s", msg);
    return NFK_EINVAL;
}

static int launch_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        std::snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
        return (int)e;
    }
    return 0;
}

extern "C" int nfk_abi_version(void) { return NFK_ABI_VERSION; }
extern "C" const char* nfk_last_error(void) { return g_err; }

NfkSplineConst nfk_make_const(int K, double left, double right, double bottom, double top,
                              int tails, double min_w, double min_h, double min_d) {
    // every constant evaluated in double as the reference's Python scalars are,
    // then rounded to fp32 once (the tensor op casts the scalar to fp32)
    NfkSplineConst c;
    c.scale2b = (float)(right - left);
    c.lo = (float)left;
    c.hi = (float)right;
    c.span = (float)(right - left);
    c.ylo = (float)bottom;
    c.yhi = (float)top;
    c.yspan = (float)(top - bottom);
    c.tails = tails ? 1 : 0;
    c.min_w = (float)min_w;
    c.fw = (float)(1.0 - min_w * K);
    c.min_h = (float)min_h;
    c.fh = (float)(1.0 - min_h * K);
    c.min_d = (float)min_d;
    c.dpad = (float)std::log(std::exp(1.0 - min_d) - 1.0);
    c.knot_eps = (float)1e-6;
    c.m2b = (float)((right - left) * 1.4426950408889634);
    c.d_edge = c.min_d + log1pf(expf(c.dpad));  // fp32 like the reference's tensor ops
    return c;
}

// ---------------------------------------------------------------------------
// wave helpers
// ---------------------------------------------------------------------------
template <int W>
__device__ __forceinline__ float group_sum(float v) {
    // deterministic butterfly over aligned groups of W lanes (W power of 2 <= 64)
#pragma unroll
    for (int off = W / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__device__ __forceinline__ void status_or(int32_t* status, int bits) {
    if (status != nullptr && bits != 0) {
        if ((__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bits) != bits)
            atomicOr(status, bits);
    }
}

// ---------------------------------------------------------------------------
// spline coupling (unfused: params come from the conditioner GEMMs in HBM)
//
// A block owns S whole samples (S = EPB / n_up, or 1 with coordinate rounds
// when n_up > EPB).  Per round the [elements, 3K-1] parameter slab -- one
// contiguous span of HBM -- is streamed into LDS with 16-B loads; each lane
// then reads its own 3K-1 params at an odd LDS stride (bank-conflict free),
// evaluates the spline in registers, and the per-sample log|det| is reduced
// in a fixed order (deterministic, no atomics).
// ---------------------------------------------------------------------------
struct RqsArgs {
    const float* x;
    int64_t ldx;
    const float* params;
    const int32_t* up_in;
    const int32_t* up_out;
    int32_t n_up;
    const int32_t* lo_in;
    const int32_t* lo_out;
    int32_t n_lo;
    float* z;
    int64_t ldz;
    float* logdet;
    int32_t logdet_mode;
    float* lad_out;
    int64_t ld_lad;
    int64_t batch;
    int32_t spb;  // samples per block
    int32_t* status;
    NfkSplineConst c;
};

// ---------------------------------------------------------------------------
// Streaming form for whole samples per round (n_up <= EPB) with 16-B aligned
// rows: a persistent grid (a few blocks per CU) walks rounds of S = EPB / n_up
// samples.  Per round the [S n_up, P] parameter slab and the S x rows are
// prefetched into registers (16-B loads) while the previous round computes,
// then stored to LDS; each lane evaluates one element from its LDS
// parameters; z rows are assembled in LDS (upper values at up_out, lower
// copies at lo_out) and written whole with 16-B stores, so every z line is
// written once.  log|det| per sample is summed in the same sequential order
// as k_rqs_coupling, and the element math is the same function, so both
// kernels give bitwise identical results.
// ---------------------------------------------------------------------------
template <int K, bool INV, bool PRE, bool DFULL, int EPB, bool LEAN>
__global__ __launch_bounds__(EPB) void k_rqs_stream(RqsArgs a, int D, int64_t nrounds) {
    constexpr int DN = NfkDN<K, DFULL>::n;
    constexpr int P = DFULL ? 3 * K + 1 : 3 * K - 1;
    constexpr int NPF = (EPB * P / 4 + EPB - 1) / EPB;  // param float4s per thread (max)
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* sp = smem;                  // [EPB][P] parameters
    float* sl = sp + EPB * P;          // [EPB] per-element log|det|
    float* sx = sl + EPB;              // [S][D] x rows
    float* sz = sx + a.spb * D;        // [S][D] z rows
    int* smap = reinterpret_cast<int*>(sz + a.spb * D);  // up_in, up_out, lo_in, lo_out
    int* cover = smap + 2 * a.n_up + 2 * a.n_lo;          // [2][D] input / output column use counts
    const int tid = threadIdx.x;
    const int S = a.spb, n_up = a.n_up, n_lo = a.n_lo, D4 = D >> 2;
    for (int i = tid; i < 2 * D; i += EPB) cover[i] = 0;
    bool bad = false;  // a map leaves the first D columns: no whole-row staging
    for (int i = tid; i < n_up; i += EPB) {
        smap[i] = a.up_in[i];
        smap[n_up + i] = a.up_out[i];
        bad |= (unsigned)a.up_in[i] >= (unsigned)D || (unsigned)a.up_out[i] >= (unsigned)D;
    }
    for (int i = tid; i < n_lo; i += EPB) {
        smap[2 * n_up + i] = a.lo_in[i];
        smap[2 * n_up + n_lo + i] = a.lo_out[i];
        bad |= (unsigned)a.lo_in[i] >= (unsigned)D || (unsigned)a.lo_out[i] >= (unsigned)D;
    }
    bad = __syncthreads_or(bad);
    // whole x and z rows only if the input maps and the output maps each hit
    // every column of [0, D) once (then x and z rows have at least D columns)
    if (!bad) {
        for (int i = tid; i < n_up; i += EPB) {
            atomicAdd(&cover[smap[i]], 1);
            atomicAdd(&cover[D + smap[n_up + i]], 1);
        }
        for (int i = tid; i < n_lo; i += EPB) {
            atomicAdd(&cover[smap[2 * n_up + i]], 1);
            atomicAdd(&cover[D + smap[2 * n_up + n_lo + i]], 1);
        }
    }
    __syncthreads();
    bool hole = false;
    if (!bad)
        for (int i = tid; i < 2 * D; i += EPB) hole |= cover[i] != 1;
    const bool rows = !__syncthreads_or(bad || hole);
    const int* m_up_in = smap;
    const int* m_up_out = smap + n_up;
    const int* m_lo_in = smap + 2 * n_up;
    const int* m_lo_out = smap + 2 * n_up + n_lo;
    const int j_el = tid % n_up, s_el = tid / n_up;  // this lane's element of a round
    typedef float v4 __attribute__((ext_vector_type(4)));  // HIP's float4 struct kept pf in scratch
    v4 pf[NPF];
    v4 xf = {0.f, 0.f, 0.f, 0.f};
    bool any_in = false, any_nd = false;  // status bits, reduced once at the end
    // prefetch round r into registers (rows past the batch are not read): the
    // register array stays in VGPRs only with this code inlined and unrolled
#define NFK_PREFETCH(RR)                                                                              \
    do {                                                                                             \
        const int64_t pb0 = (RR) * S;                                                                \
        const int pnb = (int)((a.batch - pb0) < S ? (a.batch - pb0) : S);                            \
        const v4* src = reinterpret_cast<const v4*>(a.params + pb0 * n_up * P);                      \
        const int n4 = pnb * n_up * P / 4; /* S n_up P is a multiple of 4 (host check) */            \
        /* unconditional loads (clamped index): a conditional one keeps pf out of VGPRs */           \
        _Pragma("unroll") for (int i = 0; i < NPF; ++i) {                                            \
            const int pi = i * EPB + tid;                                                            \
            pf[i] = src[pi < n4 ? pi : n4 - 1];                                                      \
        }                                                                                            \
        if (rows) {                                                                                  \
            const int t4 = tid < pnb * D4 ? tid : 0;                                                 \
            const int rr = t4 / D4, cc = t4 - rr * D4;                                               \
            xf = *reinterpret_cast<const v4*>(a.x + (pb0 + rr) * a.ldx + 4 * cc);                    \
        }                                                                                            \
    } while (0)
    int64_t r = blockIdx.x;
    if (r < nrounds) NFK_PREFETCH(r);
    for (; r < nrounds; r += gridDim.x) {
        const int64_t b0 = r * S;
        const int nb = (int)((a.batch - b0) < S ? (a.batch - b0) : S);
        const int cnt = nb * n_up;
        __syncthreads();  // the previous round's LDS reads are done (and the maps visible)
#pragma unroll
        for (int i = 0; i < NPF; ++i)
            if (i * EPB + tid < cnt * P / 4) reinterpret_cast<v4*>(sp)[i * EPB + tid] = pf[i];
        if (rows && tid < nb * D4) reinterpret_cast<v4*>(sx)[tid] = xf;
        __syncthreads();
        if (r + gridDim.x < nrounds) NFK_PREFETCH(r + gridDim.x);  // overlaps the compute below
        bool ins = false, nd = false;
        if (tid < cnt) {
            const float xv = rows ? sx[s_el * D + m_up_in[j_el]] : a.x[(b0 + s_el) * a.ldx + m_up_in[j_el]];
            float wr[K], hr[K], dr[DN];
            const float* p = sp + tid * P;
#pragma unroll
            for (int i = 0; i < K; ++i) wr[i] = p[i];
#pragma unroll
            for (int i = 0; i < K; ++i) hr[i] = p[K + i];
#pragma unroll
            for (int i = 0; i < P - 2 * K; ++i) dr[i] = p[2 * K + i];
            float out, lad;
            if constexpr (LEAN && PRE && !DFULL)
                nfk_rqs_element_lean<K, INV>(xv, wr, hr, dr, a.c, out, lad, ins, nd);
            else
                nfk_rqs_element<K, INV, PRE, DFULL>(xv, wr, hr, dr, a.c, out, lad, ins, nd);
            if (rows)
                sz[s_el * D + m_up_out[j_el]] = out;
            else
                a.z[(b0 + s_el) * a.ldz + m_up_out[j_el]] = out;
            if (a.lad_out != nullptr) a.lad_out[(b0 + s_el) * a.ld_lad + j_el] = lad;
            sl[tid] = lad;
        }
        for (int i = tid; i < nb * n_lo; i += EPB) {
            const int ss = i / n_lo, qq = i - ss * n_lo;
            if (rows)
                sz[ss * D + m_lo_out[qq]] = sx[ss * D + m_lo_in[qq]];
            else
                a.z[(b0 + ss) * a.ldz + m_lo_out[qq]] = a.x[(b0 + ss) * a.ldx + m_lo_in[qq]];
        }
        any_in |= ins;
        any_nd |= nd;
        __syncthreads();  // z rows and per-element log|det| complete
        if (rows && tid < nb * D4) {
            const int rr = tid / D4, cc = tid - rr * D4;
            *reinterpret_cast<float4*>(a.z + (b0 + rr) * a.ldz + 4 * cc) = reinterpret_cast<const float4*>(sz)[tid];
        }
        if (a.logdet_mode != 0 && tid < nb) {
            // sequential sum (k_rqs_coupling's order), read 16 B at a time
            float sum = 0.0f;
            const float* q = sl + tid * n_up;
            int i = 0;
            if ((n_up & 3) == 0)
                for (; i < n_up; i += 4) {
                    const float4 v = *reinterpret_cast<const float4*>(q + i);
                    sum += v.x;
                    sum += v.y;
                    sum += v.z;
                    sum += v.w;
                }
            for (; i < n_up; ++i) sum += q[i];
            float* dst = a.logdet + b0 + tid;
            *dst = (a.logdet_mode == 2) ? (*dst + sum) : sum;
        }
    }
    const int st_bits = (__syncthreads_or(any_in) ? NFK_ST_INSIDE_SEEN : 0) |
                        (__syncthreads_or(any_nd) ? NFK_ST_NEG_DISC : 0);
    if (tid == 0) status_or(a.status, st_bits);
#undef NFK_PREFETCH
}

template <int K, bool INV, bool PRE, bool DFULL, int EPB, bool LEAN = false>
__global__ __launch_bounds__(EPB) void k_rqs_coupling(RqsArgs a) {
    constexpr int DN = NfkDN<K, DFULL>::n;
    constexpr int P = DFULL ? 3 * K + 1 : 3 * K - 1;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* sp = smem;             // [EPB][P]
    float* sl = smem + EPB * P;   // [EPB] per-element log|det|
    const int tid = threadIdx.x;
    const int64_t b0 = (int64_t)blockIdx.x * a.spb;
    if (b0 >= a.batch) return;
    const int nb = (int)((a.batch - b0) < a.spb ? (a.batch - b0) : a.spb);
    const int64_t e_begin = b0 * a.n_up, e_end = (b0 + nb) * a.n_up;

    // identity-copied ("lower") coordinates
    for (int i = tid; i < nb * a.n_lo; i += EPB) {
        const int s = i / a.n_lo, q = i - s * a.n_lo;
        a.z[(b0 + s) * a.ldz + a.lo_out[q]] = a.x[(b0 + s) * a.ldx + a.lo_in[q]];
    }

    float run = 0.0f;  // multi-round accumulator (owner: wave 0, lane 0)
    int st_bits = 0;
    for (int64_t e0 = e_begin; e0 < e_end; e0 += EPB) {
        const int cnt = (int)((e_end - e0) < EPB ? (e_end - e0) : EPB);
        __syncthreads();  // previous round's LDS reads are done
        {
            const float* src = a.params + e0 * P;
            const int n = cnt * P;
            if ((((uintptr_t)src) & 15) == 0) {
                const int n4 = n >> 2;
                const float4* s4 = reinterpret_cast<const float4*>(src);
                for (int i = tid; i < n4; i += EPB) {
                    const float4 v = s4[i];
                    sp[4 * i + 0] = v.x;
                    sp[4 * i + 1] = v.y;
                    sp[4 * i + 2] = v.z;
                    sp[4 * i + 3] = v.w;
                }
                for (int i = (n4 << 2) + tid; i < n; i += EPB) sp[i] = src[i];
            } else {
                for (int i = tid; i < n; i += EPB) sp[i] = src[i];
            }
        }
        __syncthreads();
        bool ins = false, nd = false;
        if (tid < cnt) {
            const int64_t e = e0 + tid;
            const int64_t b = e / a.n_up;
            const int j = (int)(e - b * a.n_up);
            const float xv = a.x[b * a.ldx + a.up_in[j]];
            float wr[K], hr[K], dr[DN];
            const float* p = sp + tid * P;
#pragma unroll
            for (int i = 0; i < K; ++i) wr[i] = p[i];
#pragma unroll
            for (int i = 0; i < K; ++i) hr[i] = p[K + i];
#pragma unroll
            for (int i = 0; i < P - 2 * K; ++i) dr[i] = p[2 * K + i];
            float out, lad;
            if constexpr (LEAN && PRE && !DFULL)
                nfk_rqs_element_lean<K, INV>(xv, wr, hr, dr, a.c, out, lad, ins, nd);
            else
                nfk_rqs_element<K, INV, PRE, DFULL>(xv, wr, hr, dr, a.c, out, lad, ins, nd);
            a.z[b * a.ldz + a.up_out[j]] = out;
            if (a.lad_out != nullptr) a.lad_out[b * a.ld_lad + j] = lad;
            sl[tid] = lad;
        }
        st_bits |= (__syncthreads_or(ins) ? NFK_ST_INSIDE_SEEN : 0);
        st_bits |= (__syncthreads_or(nd) ? NFK_ST_NEG_DISC : 0);
        if (a.logdet_mode == 0) continue;
        // per-sample reduction of sl[] (the __syncthreads_or above is the barrier)
        if (a.n_up <= EPB) {
            if (a.n_up < 64) {
                if (tid < nb) {
                    float s = 0.0f;
                    const float* q = sl + tid * a.n_up;
                    for (int i = 0; i < a.n_up; ++i) s += q[i];
                    float* dst = a.logdet + b0 + tid;
                    *dst = (a.logdet_mode == 2) ? (*dst + s) : s;
                }
            } else {
                const int w = tid >> 6, lane = tid & 63;
                if (w < nb) {  // one wave per sample
                    float s = 0.0f;
                    const float* q = sl + w * a.n_up;
                    for (int i = lane; i < a.n_up; i += 64) s += q[i];
                    s = group_sum<64>(s);
                    if (lane == 0) {
                        float* dst = a.logdet + b0 + w;
                        *dst = (a.logdet_mode == 2) ? (*dst + s) : s;
                    }
                }
            }
        } else if (tid < 64) {  // one sample in coordinate rounds: wave 0 folds the round
            float s = 0.0f;
            for (int i = tid; i < cnt; i += 64) s += sl[i];
            s = group_sum<64>(s);
            run += s;
        }
    }
    if (a.n_up > EPB && a.logdet_mode != 0 && tid == 0) {
        float* dst = a.logdet + b0;
        *dst = (a.logdet_mode == 2) ? (*dst + run) : run;
    }
    if (tid == 0) status_or(a.status, st_bits);
}

// NSF_CL's raw-logit mode (PRE) runs the lean element math (nfk_rqs_element_lean,
// the fused kernel's epilogue) when the spline constants are NSF_CL's (equal x
// and y ranges, equal minimum bin width and height); NFK_RQS_LEAN=0 in the
// environment selects the reference-order math everywhere.
static bool lean_env() {
    static const bool on = [] {
        const char* e = std::getenv("NFK_RQS_LEAN");
        return !(e != nullptr && e[0] == '0');
    }();
    return on;
}

// k_rqs_stream applies when a round holds whole samples, the lower and upper
// maps cover D = n_lo + n_up columns once each (a permutation of x's and z's
// first D columns, as NSF_CL's are), and rows are 16-B aligned;
// NFK_RQS_STREAM=0 in the environment selects k_rqs_coupling everywhere.
static int g_rqs_form = -1;  // nfk_debug_rqs_form
static bool stream_env() {
    static const bool on = [] {
        const char* e = std::getenv("NFK_RQS_STREAM");
        return !(e != nullptr && e[0] == '0');
    }();
    return g_rqs_form < 0 ? on : g_rqs_form == 1;
}

// Diagnostic (not part of include/nfk.h): -1 = automatic, 0 = k_rqs_coupling
// only, 1 = k_rqs_stream where it applies.  Returns the previous setting.
extern "C" int nfk_debug_rqs_form(int form) {
    const int prev = g_rqs_form;
    g_rqs_form = form < 0 ? -1 : (form ? 1 : 0);
    return prev;
}

template <int K, bool INV, bool PRE, bool DFULL>
static int launch_rqs_k(RqsArgs a, hipStream_t st) {
    constexpr int P = DFULL ? 3 * K + 1 : 3 * K - 1;
    constexpr int EPB = (P <= 49) ? 256 : (P <= 97 ? 128 : 64);
    a.spb = a.n_up <= EPB ? EPB / a.n_up : 1;
    const int64_t blocks = (a.batch + a.spb - 1) / a.spb;
    if (blocks == 0) return 0;
    const size_t lds = (size_t)(EPB * P + EPB) * sizeof(float);
    const bool lean = PRE && !DFULL && lean_env() && a.c.ylo == a.c.lo && a.c.yhi == a.c.hi &&
                      a.c.min_w == a.c.min_h && a.c.fw == a.c.fh;
    const int D = a.n_lo + a.n_up;
    if (stream_env() && a.n_up <= EPB && D % 4 == 0 && a.ldx % 4 == 0 && a.ldz % 4 == 0 &&
        ((uintptr_t)a.x % 16) == 0 && ((uintptr_t)a.z % 16) == 0 && ((uintptr_t)a.params % 16) == 0 &&
        (a.spb * a.n_up * P) % 4 == 0 && a.spb * D / 4 <= EPB) {
        const int64_t nrounds = blocks;
        int dev = 0, ncu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
        static const int bpc = [] {  // resident blocks per CU (NFK_RQS_BPC, default 4)
            const char* e = std::getenv("NFK_RQS_BPC");
            const int v = e != nullptr ? std::atoi(e) : 4;
            return v >= 1 && v <= 16 ? v : 4;
        }();
        const int64_t grid = nrounds < (int64_t)ncu * bpc ? nrounds : (int64_t)ncu * bpc;
        const size_t lds2 = (size_t)(EPB * P + EPB + 2 * a.spb * D) * sizeof(float) +
                            (size_t)(2 * a.n_up + 2 * a.n_lo + 2 * D) * sizeof(int);
        if (lean)
            hipLaunchKernelGGL((k_rqs_stream<K, INV, PRE, DFULL, EPB, PRE && !DFULL>), dim3((unsigned)grid),
                               dim3(EPB), lds2, st, a, D, nrounds);
        else
            hipLaunchKernelGGL((k_rqs_stream<K, INV, PRE, DFULL, EPB, false>), dim3((unsigned)grid), dim3(EPB),
                               lds2, st, a, D, nrounds);
        return launch_status("nfk_rqs_coupling");
    }
    if (lean)
        hipLaunchKernelGGL((k_rqs_coupling<K, INV, PRE, DFULL, EPB, PRE && !DFULL>), dim3((unsigned)blocks),
                           dim3(EPB), lds, st, a);
    else
        hipLaunchKernelGGL((k_rqs_coupling<K, INV, PRE, DFULL, EPB>), dim3((unsigned)blocks), dim3(EPB), lds,
                           st, a);
    return launch_status("nfk_rqs_coupling");
}

template <int K>
static int launch_rqs_modes(RqsArgs a, bool inv, int mode, hipStream_t st) {
    // mode 0: NSF_CL raw (pre-normalise), 1: unconstrained_RQS args, 2: RQS args (K+1 derivs)
    if (inv) {
        if (mode == 0) return launch_rqs_k<K, true, true, false>(a, st);
        if (mode == 1) return launch_rqs_k<K, true, false, false>(a, st);
        return launch_rqs_k<K, true, false, true>(a, st);
    }
    if (mode == 0) return launch_rqs_k<K, false, true, false>(a, st);
    if (mode == 1) return launch_rqs_k<K, false, false, false>(a, st);
    return launch_rqs_k<K, false, false, true>(a, st);
}

#define NFK_RQS_KLIST(X) \
    X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(16) X(20) X(24) X(32) X(48) X(64)

extern "C" int nfk_rqs_coupling(const float* x, int64_t ldx, const float* params,
                                const int32_t* up_in, const int32_t* up_out, int32_t n_up,
                                const int32_t* lo_in, const int32_t* lo_out, int32_t n_lo,
                                float* z, int64_t ldz, float* logdet, int32_t logdet_mode,
                                float* lad_out, int64_t ld_lad, int64_t batch, int32_t K,
                                double left, double right, double bottom, double top,
                                int32_t tails, double min_bin_width, double min_bin_height,
                                double min_derivative, int32_t param_mode, int32_t inverse,
                                int32_t* status, nfk_stream_t stream) {
    if (batch < 0 || n_up <= 0 || n_lo < 0) return nfk_set_error("nfk_rqs_coupling: bad sizes");
    if (min_bin_width * K > 1.0) return nfk_set_error("Minimal bin width too large for the number of bins");
    if (min_bin_height * K > 1.0) return nfk_set_error("Minimal bin height too large for the number of bins");
    if (batch == 0) return 0;  // nothing inside: status stays 0 (reference: RuntimeError)
    if (x == nullptr || params == nullptr || z == nullptr || up_in == nullptr || up_out == nullptr)
        return nfk_set_error("nfk_rqs_coupling: null pointer");
    if (n_lo > 0 && (lo_in == nullptr || lo_out == nullptr))
        return nfk_set_error("nfk_rqs_coupling: null lower index map");
    if (logdet_mode != 0 && logdet == nullptr) return nfk_set_error("nfk_rqs_coupling: null logdet");
    RqsArgs a{x, ldx, params, up_in, up_out, n_up, lo_in, lo_out, n_lo, z, ldz, logdet,
              logdet_mode, lad_out, ld_lad, batch, 1, status,
              nfk_make_const(K, left, right, bottom, top, tails, min_bin_width, min_bin_height,
                             min_derivative)};
    if (param_mode < 0 || param_mode > 2) return nfk_set_error("nfk_rqs_coupling: bad param_mode");
    hipStream_t st = (hipStream_t)stream;
    const bool inv = inverse != 0;
    switch (K) {
#define NFK_CASE(k) \
    case k: return launch_rqs_modes<k>(a, inv, param_mode, st);
        NFK_RQS_KLIST(NFK_CASE)
#undef NFK_CASE
        default: break;
    }
    return nfk_set_error("nfk_rqs_coupling: unsupported K (supported: 2-12, 16, 20, 24, 32, 48, 64)");
}

// searchsorted (utils.py:20-25), side effect included
__global__ __launch_bounds__(256) void k_searchsorted(float* loc, const float* __restrict__ v,
                                                      int64_t* idx, int64_t rows, int n,
                                                      float eps) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows;
         r += (int64_t)gridDim.x * blockDim.x) {
        float* l = loc + r * n;
        const float last = l[n - 1] + eps;
        l[n - 1] = last;
        const float xv = v[r];
        int64_t c = 0;
        for (int j = 0; j < n - 1; ++j) c += (xv >= l[j]) ? 1 : 0;
        c += (xv >= last) ? 1 : 0;
        idx[r] = c - 1;
    }
}

extern "C" int nfk_searchsorted(float* bin_locations, const float* inputs, int64_t* idx,
                                int64_t rows, int32_t n_loc, double eps, nfk_stream_t stream) {
    if (rows < 0 || n_loc <= 0) return nfk_set_error("nfk_searchsorted: bad sizes");
    if (rows == 0) return 0;
    if (!bin_locations || !inputs || !idx) return nfk_set_error("nfk_searchsorted: null pointer");
    if (rows == 0) return 0;
    int64_t g = (rows + 255) / 256;
    if (g > 16384) g = 16384;
    hipLaunchKernelGGL(k_searchsorted, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream,
                       bin_locations, inputs, idx, rows, n_loc, (float)eps);
    return launch_status("nfk_searchsorted");
}

// ---------------------------------------------------------------------------
// row kernels: W lanes per row, 64/W rows per wave, group_sum for row sums
// ---------------------------------------------------------------------------
static inline int lanes_for(int n) {
    int w = 1;
    while (w < n && w < 64) w <<= 1;
    return w;
}

static inline unsigned grid_for_rows(int64_t rows, int w) {
    const int64_t rows_per_block = (int64_t)(256 / 64) * (64 / w);
    int64_t g = (rows + rows_per_block - 1) / rows_per_block;
    if (g > 65536) g = 65536;
    if (g < 1) g = 1;
    return (unsigned)g;
}

#define NFK_ROW_PROLOGUE(W)                                                         \
    const int lane = threadIdx.x & 63;                                              \
    const int sub = lane / (W), c0 = lane % (W);                                    \
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;      \
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;                   \
    constexpr int RPW = 64 / (W);

#define NFK_W_DISPATCH(w, CALL) \
    switch (w) {                \
        case 1: CALL(1); break; \
        case 2: CALL(2); break; \
        case 4: CALL(4); break; \
        case 8: CALL(8); break; \
        case 16: CALL(16); break; \
        case 32: CALL(32); break; \
        default: CALL(64); break; \
    }

// affine half-coupling (flows.py:56,59 forward; 69,72 inverse)
template <int W, bool INV>
__global__ __launch_bounds__(256) void k_affine(const float* __restrict__ xin, int64_t ld_in,
                                                const float* __restrict__ s,
                                                const float* __restrict__ t, int64_t ld_st,
                                                float* xout, int64_t ld_out, float* logdet,
                                                int mode, int64_t batch, int n) {
    NFK_ROW_PROLOGUE(W)
    for (int64_t r0 = wave * RPW; r0 < batch; r0 += nwave * RPW) {
        const int64_t b = r0 + sub;
        const bool ok = b < batch;
        float acc = 0.0f;
        if (ok) {
            for (int c = c0; c < n; c += W) {
                const float sv = s[b * ld_st + c], tv = t[b * ld_st + c];
                const float xv = xin[b * ld_in + c];
                float o;
                if (INV) {
                    o = (xv - tv) * expf(-sv);
                    acc += -sv;
                } else {
                    o = tv + xv * expf(sv);
                    acc += sv;
                }
                xout[b * ld_out + c] = o;
            }
        }
        acc = group_sum<W>(acc);
        if (ok && c0 == 0 && mode != 0) logdet[b] = (mode == 2) ? (logdet[b] + acc) : acc;
    }
}

extern "C" int nfk_affine_coupling(const float* x_in, int64_t ld_in, const float* s,
                                   const float* t, int64_t ld_st, float* x_out, int64_t ld_out,
                                   float* logdet, int32_t logdet_mode, int64_t batch, int32_t n,
                                   int32_t inverse, nfk_stream_t stream) {
    if (batch < 0 || n <= 0) return nfk_set_error("nfk_affine_coupling: bad sizes");
    if (batch == 0) return 0;
    if (!x_in || !s || !t || !x_out) return nfk_set_error("nfk_affine_coupling: null pointer");
    if (logdet_mode != 0 && !logdet) return nfk_set_error("nfk_affine_coupling: null logdet");
    if (batch == 0) return 0;
    const int w = lanes_for(n);
    hipStream_t st = (hipStream_t)stream;
    const unsigned g = grid_for_rows(batch, w);
#define CALL(W)                                                                               \
    if (inverse)                                                                              \
        hipLaunchKernelGGL((k_affine<W, true>), dim3(g), dim3(256), 0, st, x_in, ld_in, s, t, \
                           ld_st, x_out, ld_out, logdet, logdet_mode, batch, n);              \
    else                                                                                      \
        hipLaunchKernelGGL((k_affine<W, false>), dim3(g), dim3(256), 0, st, x_in, ld_in, s, t, \
                           ld_st, x_out, ld_out, logdet, logdet_mode, batch, n);
    NFK_W_DISPATCH(w, CALL)
#undef CALL
    return launch_status("nfk_affine_coupling");
}

// Backward of the affine half-coupling (the VJP of k_affine): per element,
//   forward  out = t + in e,  e = exp(s):   g_in = g e,  g_t = g,    g_s = g in e + g_ld
//   inverse  out = (in - t) e, e = exp(-s): g_in = g e,  g_t = -g e, g_s = -g out - g_ld
// with g = g_out (0 where null) and g_ld the row's log|det| gradient (0 where
// null).  g_in is written (acc = 0) or accumulated (acc = 1); g_t may be null
// in the forward direction (it is g_out itself).
template <int W, bool INV>
__global__ __launch_bounds__(256) void k_affine_bwd(const float* __restrict__ xin, int64_t ld_in,
                                                    const float* __restrict__ s,
                                                    const float* __restrict__ t, int64_t ld_st,
                                                    const float* __restrict__ gout, int64_t ld_g,
                                                    const float* __restrict__ gld, float* gin,
                                                    int64_t ld_gin, int acc, float* gs, float* gt,
                                                    int64_t ld_gst, int64_t batch, int n) {
    NFK_ROW_PROLOGUE(W)
    for (int64_t r0 = wave * RPW; r0 < batch; r0 += nwave * RPW) {
        const int64_t b = r0 + sub;
        if (b >= batch) continue;
        const float gl = gld ? gld[b] : 0.0f;
        for (int c = c0; c < n; c += W) {
            const float sv = s[b * ld_st + c], xv = xin[b * ld_in + c];
            const float g = gout ? gout[b * ld_g + c] : 0.0f;
            float vi, vs, vt;
            if (INV) {
                const float e = expf(-sv), o = (xv - t[b * ld_st + c]) * e;
                vi = g * e;
                vt = -g * e;
                vs = -g * o - gl;
            } else {
                const float e = expf(sv);
                vi = g * e;
                vt = g;
                vs = g * xv * e + gl;
            }
            float* pi = gin + b * ld_gin + c;
            *pi = acc ? *pi + vi : vi;
            gs[b * ld_gst + c] = vs;
            if (gt) gt[b * ld_gst + c] = vt;
        }
    }
}

extern "C" int nfk_affine_coupling_bwd(const float* x_in, int64_t ld_in, const float* s, const float* t,
                                       int64_t ld_st, const float* g_out, int64_t ld_g, const float* g_logdet,
                                       float* g_in, int64_t ld_gin, int32_t accumulate, float* g_s, float* g_t,
                                       int64_t ld_gst, int64_t batch, int32_t n, int32_t inverse,
                                       nfk_stream_t stream) {
    if (batch < 0 || n <= 0) return nfk_set_error("nfk_affine_coupling_bwd: bad sizes");
    if (batch == 0) return 0;
    if (!x_in || !s || !g_in || !g_s || (inverse && (!t || !g_t)))
        return nfk_set_error("nfk_affine_coupling_bwd: null pointer");
    const int w = lanes_for(n);
    hipStream_t st = (hipStream_t)stream;
    const unsigned g = grid_for_rows(batch, w);
#define CALL(W)                                                                                      \
    if (inverse)                                                                                     \
        hipLaunchKernelGGL((k_affine_bwd<W, true>), dim3(g), dim3(256), 0, st, x_in, ld_in, s, t, ld_st,  \
                           g_out, ld_g, g_logdet, g_in, ld_gin, accumulate, g_s, g_t, ld_gst, batch, n); \
    else                                                                                             \
        hipLaunchKernelGGL((k_affine_bwd<W, false>), dim3(g), dim3(256), 0, st, x_in, ld_in, s, t, ld_st, \
                           g_out, ld_g, g_logdet, g_in, ld_gin, accumulate, g_s, g_t, ld_gst, batch, n);
    NFK_W_DISPATCH(w, CALL)
#undef CALL
    return launch_status("nfk_affine_coupling_bwd");
}

// ---------------------------------------------------------------------------
// planar flow (flows_1.py:42-60)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float planar_h(float v, int nl) {
    if (nl == 0) return tanhf(v);
    if (nl == 1) return v > 0.0f ? v : 0.01f * v;  // F.leaky_relu(0.01)
    return v > 0.0f ? v : expm1f(v);               // F.elu(alpha=1)
}

__device__ __forceinline__ float planar_dh(float v, int nl) {
    // flows_1.py:12-18, verbatim semantics (leaky_relu's negative side is -0.01)
    if (nl == 0) {
        const float th = tanhf(v);
        return 1.0f - th * th;
    }
    const float pos = v > 0.0f ? 1.0f : 0.0f, neg = v < 0.0f ? 1.0f : 0.0f;
    if (nl == 1) return pos + neg * -0.01f;
    return pos + neg * expf(v);
}

template <int W>
__global__ __launch_bounds__(256) void k_planar(const float* __restrict__ x, int64_t ldx,
                                                const float* __restrict__ w,
                                                const float* __restrict__ u,
                                                const float* __restrict__ bp, float* z,
                                                int64_t ldz, float* logdet, int mode,
                                                float* ld_out, int64_t batch, int dim, int nl) {
    extern __shared__ __attribute__((aligned(16))) float uh[];  // [dim] u_hat
    __shared__ float red[2][4];
    // u_hat (flows_1.py:48-53), recomputed per block: dim-length dots
    {
        float wu = 0.0f, ww = 0.0f;
        for (int i = threadIdx.x; i < dim; i += blockDim.x) {
            wu += w[i] * u[i];
            ww += w[i] * w[i];
        }
        wu = group_sum<64>(wu);
        ww = group_sum<64>(ww);
        if ((threadIdx.x & 63) == 0) {
            red[0][threadIdx.x >> 6] = wu;
            red[1][threadIdx.x >> 6] = ww;
        }
        __syncthreads();
        wu = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
        ww = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
        float scal = 0.0f, nrm2 = 1.0f;
        if (nl == 0) {
            scal = logf(1.0f + expf(wu)) - wu - 1.0f;
            const float nrm = sqrtf(ww);
            nrm2 = nrm * nrm;
        }
        for (int i = threadIdx.x; i < dim; i += blockDim.x)
            uh[i] = (nl == 0) ? u[i] + (scal * w[i]) / nrm2 : u[i];
        __syncthreads();
    }
    const float bias = bp[0];
    NFK_ROW_PROLOGUE(W)
    for (int64_t r0 = wave * RPW; r0 < batch; r0 += nwave * RPW) {
        const int64_t b = r0 + sub;
        const bool ok = b < batch;
        float lin = 0.0f;
        if (ok)
            for (int c = c0; c < dim; c += W) lin += x[b * ldx + c] * w[c];
        lin = group_sum<W>(lin) + bias;
        const float hv = planar_h(lin, nl), dh = planar_dh(lin, nl);
        float pu = 0.0f;
        if (ok) {
            for (int c = c0; c < dim; c += W) {
                z[b * ldz + c] = x[b * ldx + c] + uh[c] * hv;
                pu += (dh * w[c]) * uh[c];
            }
        }
        pu = group_sum<W>(pu);
        if (ok && c0 == 0) {
            const float ld = logf(fabsf(1.0f + pu) + 1e-4f);
            if (ld_out) ld_out[b] = ld;
            if (mode != 0) logdet[b] = (mode == 2) ? (logdet[b] + ld) : ld;
        }
    }
}

extern "C" int nfk_planar(const float* x, int64_t ldx, const float* w, const float* u,
                          const float* b, float* z, int64_t ldz, float* logdet,
                          int32_t logdet_mode, float* ld_out, int64_t batch, int32_t dim,
                          int32_t nonlinearity, nfk_stream_t stream) {
    if (batch < 0 || dim <= 0 || dim > 16384) return nfk_set_error("nfk_planar: bad sizes");
    if (batch == 0) return 0;
    if (!x || !w || !u || !b || !z) return nfk_set_error("nfk_planar: null pointer");
    if (nonlinearity < 0 || nonlinearity > 2) return nfk_set_error("nfk_planar: bad nonlinearity");
    if (logdet_mode != 0 && !logdet) return nfk_set_error("nfk_planar: null logdet");
    if (batch == 0) return 0;
    const int wl = lanes_for(dim);
    hipStream_t st = (hipStream_t)stream;
    const unsigned g = grid_for_rows(batch, wl);
    const size_t lds = (size_t)dim * sizeof(float);
#define CALL(W)                                                                                \
    hipLaunchKernelGGL((k_planar<W>), dim3(g), dim3(256), lds, st, x, ldx, w, u, b, z, ldz, logdet, \
                       logdet_mode, ld_out, batch, dim, nonlinearity);
    NFK_W_DISPATCH(wl, CALL)
#undef CALL
    return launch_status("nfk_planar");
}

// ---------------------------------------------------------------------------
// radial flow (flows_1.py:85-97): batch-global norm, fixed-order fp64 reduction
// ---------------------------------------------------------------------------
static constexpr int kRadialBlocks = 1024;

extern "C" int64_t nfk_radial_workspace_elems(void) { return kRadialBlocks; }

__global__ __launch_bounds__(256) void k_radial_partial(const float* __restrict__ x, int64_t ldx,
                                                        const float* __restrict__ x0,
                                                        int64_t batch, int dim, double* ws) {
    __shared__ double red[4];
    double acc = 0.0;
    const int64_t n = batch * dim;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = i / dim;
        const int c = (int)(i - b * dim);
        const float d = x[b * ldx + c] - x0[c];
        acc += (double)d * (double)d;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) ws[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(64) void k_radial_final(const double* ws, int nb, double* out) {
    double acc = 0.0;
    for (int i = threadIdx.x; i < nb; i += 64) acc += ws[i];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (threadIdx.x == 0) *out = acc;
}

extern "C" int nfk_radial_sumsq(const float* x, int64_t ldx, const float* x0, int64_t batch,
                                int32_t dim, double* workspace, double* sumsq,
                                nfk_stream_t stream) {
    if (batch < 0 || dim <= 0) return nfk_set_error("nfk_radial_sumsq: bad sizes");
    if (!x || !x0 || !workspace || !sumsq) return nfk_set_error("nfk_radial_sumsq: null pointer");
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_radial_partial, dim3(kRadialBlocks), dim3(256), 0, st, x, ldx, x0, batch,
                       dim, workspace);
    hipLaunchKernelGGL(k_radial_final, dim3(1), dim3(64), 0, st, workspace, kRadialBlocks, sumsq);
    return launch_status("nfk_radial_sumsq");
}

__global__ __launch_bounds__(256) void k_radial_apply(const float* __restrict__ x, int64_t ldx,
                                                      const float* __restrict__ x0,
                                                      const float* la, const float* be,
                                                      const double* sumsq, float* z, int64_t ldz,
                                                      float* ld_scalar, float* logdet, int mode,
                                                      int64_t batch, int dim) {
    const float r = (float)sqrt(*sumsq);
    const float ea = expf(la[0]);
    const float h = 1.0f / (ea + r);
    const float bh = -ea + logf(1.0f + expf(be[0]));
    const float bhh = bh * h;
    const float ear = ea + r;
    const float ld = (float)(dim - 1) * logf(1.0f + bhh) + logf((1.0f + bhh) - (bh * r) / (ear * ear));
    if (blockIdx.x == 0 && threadIdx.x == 0 && ld_scalar) ld_scalar[0] = ld;
    const int64_t n = batch * dim;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = i / dim;
        const int c = (int)(i - b * dim);
        const float xv = x[b * ldx + c];
        z[b * ldz + c] = xv + bhh * (xv - x0[c]);
        if (c == 0 && mode != 0) logdet[b] = (mode == 2) ? (logdet[b] + ld) : ld;
    }
}

extern "C" int nfk_radial_apply(const float* x, int64_t ldx, const float* x0,
                                const float* log_alpha, const float* beta, const double* sumsq,
                                float* z, int64_t ldz, float* ld_scalar, float* logdet,
                                int32_t logdet_mode, int64_t batch, int32_t dim,
                                nfk_stream_t stream) {
    if (batch < 0 || dim <= 0) return nfk_set_error("nfk_radial_apply: bad sizes");
    if (!x || !x0 || !log_alpha || !beta || !sumsq || !z)
        return nfk_set_error("nfk_radial_apply: null pointer");
    if (logdet_mode != 0 && !logdet) return nfk_set_error("nfk_radial_apply: null logdet");
    hipStream_t st = (hipStream_t)stream;
    int64_t g = (batch * dim + 255) / 256;
    if (g > 16384) g = 16384;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(k_radial_apply, dim3((unsigned)g), dim3(256), 0, st, x, ldx, x0, log_alpha,
                       beta, sumsq, z, ldz, ld_scalar, logdet, logdet_mode, batch, dim);
    return launch_status("nfk_radial_apply");
}

// ---------------------------------------------------------------------------
// isotropic normal prior epilogue (torch MultivariateNormal(0, var*I).log_prob)
// ---------------------------------------------------------------------------
template <int W>
__global__ __launch_bounds__(256) void k_normal_lp(const float* __restrict__ z, int64_t ldz,
                                                   const float* __restrict__ logdet, float* out,
                                                   int64_t batch, int dim, float lii, float c2pi,
                                                   float hld, int sign, int32_t* status) {
    NFK_ROW_PROLOGUE(W)
    for (int64_t r0 = wave * RPW; r0 < batch; r0 += nwave * RPW) {
        const int64_t b = r0 + sub;
        const bool ok = b < batch;
        float m = 0.0f;
        if (ok)
            for (int c = c0; c < dim; c += W) {
                const float y = z[b * ldz + c] / lii;  // triangular solve with L = sqrt(var) I
                m += y * y;
            }
        m = group_sum<W>(m);
        if (ok && c0 == 0) {
            float lp = -0.5f * (c2pi + m) - hld;
            if (logdet) lp = (sign >= 0) ? (lp + logdet[b]) : (lp - logdet[b]);
            out[b] = lp;
        }
        // a NaN in the row makes m NaN (squares of infinities stay infinite)
        if (__any(ok && c0 == 0 && m != m) && status != nullptr && (threadIdx.x & 63) == 0)
            atomicOr(status, NFK_ST_NAN_Z);
    }
}

// float4 form for dim % 4 == 0 and 16-B aligned rows: one 16-B load per lane
// per step; y = z * (1/L) instead of the solve's z / L (<= 1 ulp per element)
template <int W>
__global__ __launch_bounds__(256) void k_normal_lp4(const float4* __restrict__ z4, int64_t ldz4,
                                                    const float* __restrict__ logdet, float* out,
                                                    int64_t batch, int dim4, float inv_l, float c2pi,
                                                    float hld, int sign, int32_t* status) {
    NFK_ROW_PROLOGUE(W)
    for (int64_t r0 = wave * RPW; r0 < batch; r0 += nwave * RPW) {
        const int64_t b = r0 + sub;
        const bool ok = b < batch;
        float m = 0.0f;
        if (ok)
            for (int c = c0; c < dim4; c += W) {
                const float4 v = z4[b * ldz4 + c];
                const float y0 = v.x * inv_l, y1 = v.y * inv_l, y2 = v.z * inv_l, y3 = v.w * inv_l;
                m += (y0 * y0 + y1 * y1) + (y2 * y2 + y3 * y3);
            }
        m = group_sum<W>(m);
        if (ok && c0 == 0) {
            float lp = -0.5f * (c2pi + m) - hld;
            if (logdet) lp = (sign >= 0) ? (lp + logdet[b]) : (lp - logdet[b]);
            out[b] = lp;
        }
        // a NaN in the row makes m NaN (squares of infinities stay infinite)
        if (__any(ok && c0 == 0 && m != m) && status != nullptr && (threadIdx.x & 63) == 0)
            atomicOr(status, NFK_ST_NAN_Z);
    }
}

extern "C" int nfk_normal_logprob(const float* z, int64_t ldz, const float* logdet, float* out,
                                  int64_t batch, int32_t dim, float scale, float half_log_det,
                                  int32_t sign, int32_t* status, nfk_stream_t stream) {
    if (batch < 0 || dim <= 0 || !(scale > 0.0f)) return nfk_set_error("nfk_normal_logprob: bad args");
    if (batch == 0) return 0;
    if (!z || !out) return nfk_set_error("nfk_normal_logprob: null pointer");
    if (batch == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const float lii = scale;
    const float c2pi = (float)(dim * std::log(2.0 * M_PI));
    if (dim % 4 == 0 && ldz % 4 == 0 && ((uintptr_t)z & 15) == 0) {
        const int dim4 = dim / 4, w4 = lanes_for(dim4);
        const unsigned g4 = grid_for_rows(batch, w4);
        const float inv_l = 1.0f / lii;
#define CALL4(W)                                                                                   \
    hipLaunchKernelGGL((k_normal_lp4<W>), dim3(g4), dim3(256), 0, st, (const float4*)z, ldz / 4, logdet, \
                       out, batch, dim4, inv_l, c2pi, half_log_det, sign, status);
        NFK_W_DISPATCH(w4, CALL4)
#undef CALL4
        return launch_status("nfk_normal_logprob");
    }
    const int w = lanes_for(dim);
    const unsigned g = grid_for_rows(batch, w);
#define CALL(W)                                                                                 \
    hipLaunchKernelGGL((k_normal_lp<W>), dim3(g), dim3(256), 0, st, z, ldz, logdet, out, batch, dim, \
                       lii, c2pi, half_log_det, sign, status);
    NFK_W_DISPATCH(w, CALL)
#undef CALL
    return launch_status("nfk_normal_logprob");
}

// ---------------------------------------------------------------------------
// NSF_AR trig features (flows.py:172-173)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_trig(const float* __restrict__ x, int64_t ldx, float* f,
                                              int64_t ldf, int64_t batch, int n, float pi,
                                              float bnd) {
    const int64_t tot = batch * n;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < tot;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = i / n;
        const int c = (int)(i - b * n);
        const float a = (pi * x[b * ldx + c]) / bnd;
        f[b * ldf + c] = cosf(a);
        f[b * ldf + n + c] = sinf(a);
    }
}

extern "C" int nfk_trig_features(const float* x, int64_t ldx, float* feat, int64_t ldf,
                                 int64_t batch, int32_t n, double B, nfk_stream_t stream) {
    if (batch < 0 || n <= 0) return nfk_set_error("nfk_trig_features: bad sizes");
    if (batch == 0) return 0;
    if (!x || !feat) return nfk_set_error("nfk_trig_features: null pointer");
    if (batch == 0) return 0;
    int64_t g = (batch * n + 255) / 256;
    if (g > 16384) g = 16384;
    hipLaunchKernelGGL(k_trig, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, x, ldx, feat,
                       ldf, batch, n, (float)M_PI, (float)B);
    return launch_status("nfk_trig_features");
}
