// nfk_flows_extra.hip -- elementwise steps of the remaining flow classes of
// nf/flows_1.py: MAF's per-coordinate affine map and
// ActNorm.  HBM-bound row kernels, one pass over x and z.  Built with
// -ffp-contract=off like the other streaming kernels, so each fp32 op rounds
// as the reference's ATen op does.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../../include/nfk.h"

int nfk_set_error(const char* msg);

namespace {

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

unsigned grid_for(int64_t items, int per_block) {
    int64_t g = (items + per_block - 1) / per_block;
    if (g > 65536) g = 65536;
    return (unsigned)(g < 1 ? 1 : g);
}

// MAF (flows_1.py:171-195).  One lane per sample walks the columns in order,
// so the per-sample log|det| accumulates in the reference's order.
//   forward: out[b, dim-1-i] = (x[b, i] - mu_i) / exp(alpha_i);  ld -= alpha_i
//   inverse: out[b, i] = mu_i + exp(alpha_i) * x[b, dim-1-i];    ld += alpha_i
// (mu_0, alpha_0) = init[0..1]; for i >= 1 the pair is prm[b*ldp + 2*(i - p0)],
// p0 = max(c0, 1): the conditioner outputs of the columns in [max(c0,1), c1).
__global__ __launch_bounds__(256) void k_maf(const float* __restrict__ x, int64_t ldx,
                                             const float* __restrict__ init,
                                             const float* __restrict__ prm, int64_t ldp, int c0,
                                             int c1, int dim, float* out, int64_t ldo,
                                             float* logdet, int mode, int64_t batch, int inv) {
    const int p0 = c0 > 1 ? c0 : 1;
    const float mu0 = init[0], al0 = init[1];
    for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < batch;
         b += (int64_t)gridDim.x * blockDim.x) {
        float ld = 0.0f;
        for (int i = c0; i < c1; ++i) {
            float mu = mu0, al = al0;
            if (i > 0) {
                mu = prm[b * ldp + 2 * (i - p0)];
                al = prm[b * ldp + 2 * (i - p0) + 1];
            }
            if (inv) {
                out[b * ldo + i] = mu + expf(al) * x[b * ldx + (dim - 1 - i)];
                ld = ld + al;
            } else {
                out[b * ldo + (dim - 1 - i)] = (x[b * ldx + i] - mu) / expf(al);
                ld = ld - al;
            }
        }
        if (mode != 0) logdet[b] = (mode == 2) ? (logdet[b] + ld) : ld;
    }
}

// ActNorm (flows_1.py:207-215): z = x * exp(log_sigma) + mu, log|det| =
// sum(log_sigma) (a scalar, broadcast over the batch); inverse
// x = (z - mu) / exp(log_sigma), -sum(log_sigma).
template <int W>
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = W / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__global__ __launch_bounds__(256) void k_actnorm(const float* __restrict__ x, int64_t ldx,
                                                 const float* __restrict__ mu,
                                                 const float* __restrict__ ls, int dim,
                                                 float* z, int64_t ldz, float* logdet, int mode,
                                                 float* ld_scalar, int64_t batch, int inv) {
    // every wave forms the scalar in the same fixed order
    const int lane = threadIdx.x & 63;
    float s = 0.0f;
    for (int c = lane; c < dim; c += 64) s += ls[c];
    s = wave_sum<64>(s);
    const float ldv = inv ? -s : s;
    if (ld_scalar != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *ld_scalar = ldv;
    const int64_t total = batch * (int64_t)dim;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = e / dim;
        const int c = (int)(e - b * dim);
        const float v = x[b * ldx + c];
        z[b * ldz + c] = inv ? (v - mu[c]) / expf(ls[c]) : v * expf(ls[c]) + mu[c];
        if (c == 0 && mode != 0) logdet[b] = (mode == 2) ? (logdet[b] + ldv) : ldv;
    }
}

}  // namespace

extern "C" int nfk_maf(const float* x, int64_t ldx, const float* init_param, const float* params,
                       int64_t ldp, int32_t c0, int32_t c1, int32_t dim, float* out, int64_t ldo,
                       float* logdet, int32_t logdet_mode, int64_t batch, int32_t inverse,
                       nfk_stream_t stream) {
    if (batch < 0 || dim <= 0 || c0 < 0 || c1 > dim || c0 > c1) return nfk_set_error("nfk_maf: bad sizes");
    if (batch == 0 || c0 == c1) return 0;
    if (!x || !init_param || !out) return nfk_set_error("nfk_maf: null pointer");
    if (c1 > 1 && !params) return nfk_set_error("nfk_maf: null conditioner output");
    if (logdet_mode != 0 && !logdet) return nfk_set_error("nfk_maf: null logdet");
    hipLaunchKernelGGL(k_maf, dim3(grid_for(batch, 256)), dim3(256), 0, (hipStream_t)stream, x,
                       ldx, init_param, params, ldp, c0, c1, dim, out, ldo, logdet, logdet_mode,
                       batch, inverse);
    return launch_status("nfk_maf");
}

extern "C" int nfk_actnorm(const float* x, int64_t ldx, const float* mu, const float* log_sigma,
                           int32_t dim, float* z, int64_t ldz, float* logdet, int32_t logdet_mode,
                           float* ld_scalar, int64_t batch, int32_t inverse, nfk_stream_t stream) {
    if (batch < 0 || dim <= 0) return nfk_set_error("nfk_actnorm: bad sizes");
    if (!mu || !log_sigma) return nfk_set_error("nfk_actnorm: null pointer");
    if (batch > 0 && (!x || !z)) return nfk_set_error("nfk_actnorm: null pointer");
    if (logdet_mode != 0 && !logdet) return nfk_set_error("nfk_actnorm: null logdet");
    hipLaunchKernelGGL(k_actnorm, dim3(grid_for(batch * (int64_t)dim, 256)), dim3(256), 0,
                       (hipStream_t)stream, x, ldx, mu, log_sigma, dim, z, ldz, logdet,
                       logdet_mode, ld_scalar, batch, inverse);
    return launch_status("nfk_actnorm");
}
