// nfk_flows_bwd.hip -- training backward (vector-Jacobian products) of the
// flow classes outside the coupling hot path: Planar and Radial
// (nf/flows_1.py:21-97), ActNorm (flows_1.py:198-215), MAF's per-coordinate
// affine step (flows_1.py:159-195) and the NSF_AR trig features
// (nf/flows.py:172-173).  The conditioner networks of MAF / NSF_AR are
// differentiated by the host (fcnn_grad: GEMMs); everything per element and
// every batch reduction is here.
//
// Batch reductions (parameter gradients are sums over the batch) go through
// one deterministic column-sum: row chunks in a fixed order, fp64
// accumulation, partials in the caller's workspace, then a fixed-order sum of
// the chunks.  No float atomics, so a gradient is bitwise reproducible.
//
// HBM-bound row kernels; built with -ffp-contract=off like the forward ones.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

#include "../../include/nfk.h"

int nfk_set_error(const char* msg);

namespace {

constexpr int kColChunks = 128;  // row chunks of a column reduction

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

// ---- workspace: [colsum partials: kColChunks * dim doubles][row scalars:
// 3 * batch floats][sums: 3 * dim + 8 floats]
struct Ws {
    double* part;
    float* rows;
    float* sums;
};
size_t ws_bytes(int64_t batch, int dim) {
    const size_t a = (size_t)kColChunks * (size_t)(dim > 2 ? dim : 2) * sizeof(double);
    const size_t b = (size_t)(3 * batch + 4) * sizeof(float);
    const size_t c = (size_t)(3 * (int64_t)dim + 8) * sizeof(float);
    return ((a + 255) / 256 + (b + 255) / 256 + (c + 255) / 256) * 256;
}
Ws ws_carve(void* p, int64_t batch, int dim) {
    char* c = static_cast<char*>(p);
    Ws w;
    w.part = reinterpret_cast<double*>(c);
    c += ((size_t)kColChunks * (size_t)(dim > 2 ? dim : 2) * sizeof(double) + 255) / 256 * 256;
    w.rows = reinterpret_cast<float*>(c);
    c += ((size_t)(3 * batch + 4) * sizeof(float) + 255) / 256 * 256;
    w.sums = reinterpret_cast<float*>(c);
    return w;
}

// part[ch * dim + c] = sum over the rows of chunk ch of v[r] * A[r, c] * Bm[r, c]
// (v, Bm nullable = 1).  64 columns per block, its 4 waves take every 4th row.
__global__ __launch_bounds__(256) void k_colsum_part(const float* __restrict__ A, int64_t lda,
                                                     const float* __restrict__ Bm, int64_t ldb,
                                                     const float* __restrict__ v, int64_t batch, int dim,
                                                     int64_t rows_per_chunk, double* part) {
    __shared__ double red[4][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane;
    const int64_t ch = blockIdx.y;
    const int64_t r0 = ch * rows_per_chunk;
    const int64_t r1 = (r0 + rows_per_chunk < batch) ? r0 + rows_per_chunk : batch;
    double acc = 0.0;
    if (c < dim) {
        for (int64_t r = r0 + wv; r < r1; r += 4) {
            double t = (double)A[r * lda + c];
            if (Bm != nullptr) t *= (double)Bm[r * ldb + c];
            if (v != nullptr) t *= (double)v[r];
            acc += t;
        }
    }
    red[wv][lane] = acc;
    __syncthreads();
    if (wv == 0 && c < dim) part[ch * dim + c] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

__global__ __launch_bounds__(256) void k_colsum_final(const double* __restrict__ part, int nch, int dim,
                                                      float* out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= dim) return;
    double s = 0.0;
    for (int ch = 0; ch < nch; ++ch) s += part[(int64_t)ch * dim + c];
    out[c] = (float)s;
}

// out[c] = sum_b v[b] A[b, c] Bm[b, c], c < dim
void colsum(const float* A, int64_t lda, const float* Bm, int64_t ldb, const float* v, int64_t batch, int dim,
            double* part, float* out, hipStream_t st) {
    int nch = 0;
    int64_t per = 1;
    if (batch > 0) {
        nch = (int)((batch + 255) / 256);
        if (nch > kColChunks) nch = kColChunks;
        per = (batch + nch - 1) / nch;
        nch = (int)((batch + per - 1) / per);
        hipLaunchKernelGGL(k_colsum_part, dim3((unsigned)((dim + 63) / 64), (unsigned)nch), dim3(256), 0, st, A,
                           lda, Bm, ldb, v, batch, dim, per, part);
    }
    hipLaunchKernelGGL(k_colsum_final, dim3((unsigned)((dim + 255) / 256)), dim3(256), 0, st, part, nch, dim, out);
}

// fixed-order block sum of one value per thread (blockDim.x == 256)
__device__ double block_sum(double v, double* red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}

template <int W>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
    for (int off = W / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// ---------------------------------------------------------------------------
// Planar (flows_1.py:42-60): z = x + u_hat h(lin), lin = x.w + b,
// log|det| = log(|1 + h'(lin) w.u_hat| + 1e-4) with h' the reference's
// functional_derivatives (flows_1.py:12-18, leaky_relu's negative side -0.01).
// Per row, with s = 1 + dh w.u_hat and c = gld sign(s) / (|s| + 1e-4):
//   dL/dlin = a'(lin) (gz.u_hat) + c dh'(lin) w.u_hat      (a' = true h')
//   gx = gz + dL/dlin w
// and the batch sums  Gw = sum dL/dlin x,  Gu = sum h(lin) gz,
// Gb = sum dL/dlin,  C1 = sum c dh  give the parameter gradients.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void planar_fns(float lin, int nl, float& a, float& ap, float& dh, float& d2h) {
    if (nl == 0) {
        const float th = tanhf(lin);
        a = th;
        ap = 1.0f - th * th;
        dh = 1.0f - th * th;
        d2h = -2.0f * th * (1.0f - th * th);
    } else if (nl == 1) {
        a = lin > 0.0f ? lin : 0.01f * lin;           // F.leaky_relu
        ap = lin > 0.0f ? 1.0f : 0.01f;               // its autograd derivative
        dh = (lin > 0.0f ? 1.0f : 0.0f) + (lin < 0.0f ? 1.0f : 0.0f) * -0.01f;
        d2h = 0.0f;                                   // the masks carry no gradient
    } else {
        const float e = expf(lin);
        a = lin > 0.0f ? lin : e - 1.0f;              // F.elu, alpha 1
        ap = lin > 0.0f ? 1.0f : e;
        dh = (lin > 0.0f ? 1.0f : 0.0f) + (lin < 0.0f ? 1.0f : 0.0f) * e;
        d2h = lin < 0.0f ? e : 0.0f;
    }
}

// u_hat (flows_1.py:48-53) into LDS, and w.u_hat; every block recomputes it
__device__ float planar_uhat(const float* w, const float* u, int dim, int nl, float* uh, double* red) {
    double wu = 0.0, ww = 0.0;
    for (int i = threadIdx.x; i < dim; i += blockDim.x) {
        wu += (double)(w[i] * u[i]);
        ww += (double)(w[i] * w[i]);
    }
    const float fwu = (float)block_sum(wu, red);
    const float fww = (float)block_sum(ww, red);
    float scal = 0.0f, nrm2 = 1.0f;
    if (nl == 0) {
        scal = logf(1.0f + expf(fwu)) - fwu - 1.0f;
        const float nrm = sqrtf(fww);
        nrm2 = nrm * nrm;
    }
    double wuh = 0.0;
    for (int i = threadIdx.x; i < dim; i += blockDim.x) {
        const float v = (nl == 0) ? u[i] + (scal * w[i]) / nrm2 : u[i];
        uh[i] = v;
        wuh += (double)(w[i] * v);
    }
    return (float)block_sum(wuh, red);  // its barriers also publish uh
}

template <int W>
__global__ __launch_bounds__(256) void k_planar_bwd_rows(const float* __restrict__ x, int64_t ldx,
                                                         const float* __restrict__ w, const float* __restrict__ u,
                                                         const float* __restrict__ bp, const float* __restrict__ gz,
                                                         int64_t ldgz, const float* __restrict__ gld, float* gx,
                                                         int64_t ldgx, float* rows, int64_t batch, int dim, int nl) {
    extern __shared__ __attribute__((aligned(16))) float uh[];
    __shared__ double red[4];
    const float wuh = planar_uhat(w, u, dim, nl, uh, red);
    const float bias = bp[0];
    const int lane = threadIdx.x & 63;
    const int sub = lane / W, c0 = lane % W;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    constexpr int RPW = 64 / W;
    for (int64_t r0 = wave * RPW; r0 < batch; r0 += nwave * RPW) {
        const int64_t b = r0 + sub;
        const bool ok = b < batch;
        float lin = 0.0f, gu = 0.0f;
        if (ok)
            for (int c = c0; c < dim; c += W) {
                lin += x[b * ldx + c] * w[c];
                if (gz != nullptr) gu += gz[b * ldgz + c] * uh[c];
            }
        lin = group_sum<W>(lin) + bias;
        gu = group_sum<W>(gu);
        float a, ap, dh, d2h;
        planar_fns(lin, nl, a, ap, dh, d2h);
        const float s = 1.0f + dh * wuh;
        const float g = (ok && gld != nullptr) ? gld[b] : 0.0f;
        const float sg = s > 0.0f ? 1.0f : (s < 0.0f ? -1.0f : 0.0f);
        const float cc = g * sg / (fabsf(s) + 1e-4f);
        const float dlin = ap * gu + cc * d2h * wuh;
        if (ok) {
            for (int c = c0; c < dim; c += W)
                gx[b * ldgx + c] = (gz != nullptr ? gz[b * ldgz + c] : 0.0f) + dlin * w[c];
            if (c0 == 0) {
                rows[b] = dlin;
                rows[batch + b] = a;
                rows[2 * batch + b] = cc * dh;
            }
        }
    }
}

// parameter gradients from the batch sums S = [Gw (dim), Gu (dim), Gb, C1]
// (one block): through w.u_hat, then the tanh re-parameterisation of u
__global__ __launch_bounds__(256) void k_planar_bwd_params(const float* __restrict__ w, const float* __restrict__ u,
                                                           const float* __restrict__ S, float* gw, float* gu, float* gb,
                                                           int dim, int nl) {
    __shared__ double red[4];
    const float C1 = S[2 * dim + 1];
    double wu = 0.0, ww = 0.0;
    for (int i = threadIdx.x; i < dim; i += blockDim.x) {
        wu += (double)(w[i] * u[i]);
        ww += (double)(w[i] * w[i]);
    }
    const float fwu = (float)block_sum(wu, red);
    const float fww = (float)block_sum(ww, red);
    float m = 0.0f, n2 = 1.0f, sig = 0.0f;
    if (nl == 0) {
        m = logf(1.0f + expf(fwu)) - fwu - 1.0f;
        const float nrm = sqrtf(fww);
        n2 = nrm * nrm;
        sig = 1.0f / (1.0f + expf(-fwu));
    }
    // guh = Gu + C1 w;  A = sum guh w
    double A = 0.0;
    for (int i = threadIdx.x; i < dim; i += blockDim.x) A += (double)((S[dim + i] + C1 * w[i]) * w[i]);
    const float fA = (float)block_sum(A, red);
    for (int i = threadIdx.x; i < dim; i += blockDim.x) {
        const float uhi = (nl == 0) ? u[i] + (m * w[i]) / n2 : u[i];
        const float guh = S[dim + i] + C1 * w[i];
        float gwi = S[i] + C1 * uhi;
        float gui = guh;
        if (nl == 0) {
            const float k = (fA / n2) * (sig - 1.0f);
            gui = guh + k * w[i];
            gwi += k * u[i] + (m * guh) / n2 - (2.0f * m * w[i] * fA) / (n2 * n2);
        }
        gw[i] = gwi;
        gu[i] = gui;
    }
    if (threadIdx.x == 0) gb[0] = S[2 * dim];
}

// ---------------------------------------------------------------------------
// ActNorm (flows_1.py:207-215)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_actnorm_bwd_x(const float* __restrict__ gz, int64_t ldgz,
                                                       const float* __restrict__ ls, int dim, float* gx, int64_t ldgx,
                                                       int64_t batch, int inv) {
    const int64_t total = batch * (int64_t)dim;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = e / dim;
        const int c = (int)(e - b * dim);
        const float g = gz[b * ldgz + c];
        gx[b * ldgx + c] = inv ? g / expf(ls[c]) : g * expf(ls[c]);
    }
}

// S = [sum gz (dim), sum gz x (dim)]
__global__ __launch_bounds__(256) void k_actnorm_bwd_params(const float* __restrict__ mu, const float* __restrict__ ls,
                                                            const float* __restrict__ S, const float* gld, int dim,
                                                            float* gmu, float* gls, int inv) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= dim) return;
    const float g = gld != nullptr ? gld[0] : 0.0f;
    const float e = expf(ls[c]);
    if (!inv) {
        gmu[c] = S[c];
        gls[c] = e * S[dim + c] + g;
    } else {
        gmu[c] = -S[c] / e;
        gls[c] = -(S[dim + c] - mu[c] * S[c]) / e - g;
    }
}

// ---------------------------------------------------------------------------
// Radial (flows_1.py:85-97): r = sqrt(sumsq) is batch-global.  With
// G = sum_{b,c} gz (x - x0), A = 1 + bh h, C = 1 + bh h - bh r h^2:
//   dL/dbh = g ((n-1) h/A + (h - r h^2)/C) + G h
//   dL/dh  = g ((n-1) bh/A + (bh - 2 bh r h)/C) + G bh
//   dL/dr  = -g bh h^2 / C - dL/dh h^2,   dL/dsumsq = dL/dr / (2r)
//   dL/dlog_alpha = (-dL/dh h^2 - dL/dbh) e^la,  dL/dbeta = dL/dbh sigmoid(beta)
// scal = [dL/dsumsq, dL/dlog_alpha, dL/dbeta, bh h]; S = [Gz, Gzx, Xs]
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_radial_bwd_scalars(const float* __restrict__ x0, const float* la_p,
                                                            const float* be_p, const double* sumsq,
                                                            const float* __restrict__ S, const float* gld, int dim,
                                                            float* scal) {
    __shared__ double red[4];
    double G = 0.0;
    for (int c = threadIdx.x; c < dim; c += blockDim.x) G += (double)S[dim + c] - (double)x0[c] * (double)S[c];
    const double Gs = block_sum(G, red);
    if (threadIdx.x != 0) return;
    const double g = gld != nullptr ? (double)gld[0] : 0.0;
    const double r = sqrt(*sumsq);
    const double ea = exp((double)la_p[0]);
    const double be = (double)be_p[0];
    const double h = 1.0 / (ea + r);
    const double bh = -ea + log1p(exp(be));
    const double A = 1.0 + bh * h;
    const double C = 1.0 + bh * h - bh * r * h * h;
    const double n1 = (double)(dim - 1);
    const double L_bh = g * (n1 * h / A + (h - r * h * h) / C) + Gs * h;
    const double L_h = g * (n1 * bh / A + (bh - 2.0 * bh * r * h) / C) + Gs * bh;
    const double L_r = -g * bh * h * h / C - L_h * h * h;
    scal[0] = (float)(L_r / (2.0 * r));
    scal[1] = (float)((-L_h * h * h - L_bh) * ea);
    scal[2] = (float)(L_bh / (1.0 + exp(-be)));
    // bh h as the forward forms it (fp32, k_radial_apply)
    const float fr = (float)sqrt(*sumsq);
    const float fea = expf(la_p[0]);
    const float fh = 1.0f / (fea + fr);
    const float fbh = -fea + logf(1.0f + expf(be_p[0]));
    scal[3] = fbh * fh;
}

// gx = gz (1 + bh h) + 2 dL/dsumsq (x - x0); block 0 also writes
// g_x0 = -bh h Gz - 2 dL/dsumsq (Xs - batch x0)
__global__ __launch_bounds__(256) void k_radial_bwd_apply(const float* __restrict__ x, int64_t ldx,
                                                          const float* __restrict__ x0, const float* __restrict__ gz,
                                                          int64_t ldgz, const float* __restrict__ scal,
                                                          const float* __restrict__ S, float* gx, int64_t ldgx,
                                                          float* gx0, int64_t batch, int dim) {
    const float Lsq = scal[0], bhh = scal[3];
    const int64_t total = batch * (int64_t)dim;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = e / dim;
        const int c = (int)(e - b * dim);
        const float xv = x[b * ldx + c];
        const float g = gz != nullptr ? gz[b * ldgz + c] : 0.0f;
        gx[b * ldgx + c] = g * (1.0f + bhh) + 2.0f * Lsq * (xv - x0[c]);
    }
    if (blockIdx.x == 0 && gx0 != nullptr)
        for (int c = threadIdx.x; c < dim; c += blockDim.x)
            gx0[c] = -bhh * S[c] - 2.0f * Lsq * (S[2 * dim + c] - (float)batch * x0[c]);
}

// ---------------------------------------------------------------------------
// MAF per-coordinate affine step (flows_1.py:171-195), columns [c0, c1):
//   forward  o = (x_i - mu)/e^al at out column dim-1-i:
//            gx_i = go / e^al,  gmu = -go / e^al,  gal = -go o - gld
//   inverse  o = mu + e^al x_{dim-1-i} at out column i:
//            gx_{dim-1-i} = go e^al,  gmu = go,  gal = go e^al x_{dim-1-i} + gld
// (mu, al) of column 0 are init_param: their per-row gradients go to
// ginit_rows [batch, 2] (summed over the batch by the caller's colsum);
// the others to gparams[b*ldgp + 2*(i - max(c0,1)) + {0,1}].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_maf_bwd(const float* __restrict__ x, int64_t ldx,
                                                 const float* __restrict__ init, const float* __restrict__ prm,
                                                 int64_t ldp, const float* __restrict__ gout, int64_t ldgo,
                                                 const float* __restrict__ gld, int c0, int c1, int dim, float* gx,
                                                 int64_t ldgx, float* gprm, int64_t ldgp, float* ginit_rows,
                                                 int64_t batch, int inv) {
    const int p0 = c0 > 1 ? c0 : 1;
    for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < batch;
         b += (int64_t)gridDim.x * blockDim.x) {
        const float g = gld != nullptr ? gld[b] : 0.0f;
        for (int i = c0; i < c1; ++i) {
            float mu = init[0], al = init[1];
            if (i > 0) {
                mu = prm[b * ldp + 2 * (i - p0)];
                al = prm[b * ldp + 2 * (i - p0) + 1];
            }
            const float e = expf(al);
            float gmu, gal;
            if (inv) {
                const float go = gout != nullptr ? gout[b * ldgo + i] : 0.0f;
                const float xv = x[b * ldx + (dim - 1 - i)];
                gx[b * ldgx + (dim - 1 - i)] = go * e;
                gmu = go;
                gal = go * e * xv + g;
            } else {
                const float go = gout != nullptr ? gout[b * ldgo + (dim - 1 - i)] : 0.0f;
                const float o = (x[b * ldx + i] - mu) / e;
                gx[b * ldgx + i] = go / e;
                gmu = -go / e;
                gal = -go * o - g;
            }
            if (i == 0) {
                ginit_rows[2 * b] = gmu;
                ginit_rows[2 * b + 1] = gal;
            } else {
                gprm[b * ldgp + 2 * (i - p0)] = gmu;
                gprm[b * ldgp + 2 * (i - p0) + 1] = gal;
            }
        }
    }
}

// NSF_AR trig features (flows.py:172-173): feat = [cos(pi x / B), sin(pi x / B)]
//   gx[b, j] += (pi / B) (-sin(a) gfeat[b, j] + cos(a) gfeat[b, n + j]),  a = pi x / B
__global__ __launch_bounds__(256) void k_trig_bwd(const float* __restrict__ x, int64_t ldx,
                                                  const float* __restrict__ gf, int64_t ldgf, float* gx, int64_t ldgx,
                                                  int64_t batch, int n, float pi, float bnd) {
    const int64_t total = batch * (int64_t)n;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = i / n;
        const int c = (int)(i - b * n);
        const float a = (pi * x[b * ldx + c]) / bnd;
        const float d = -sinf(a) * gf[b * ldgf + c] + cosf(a) * gf[b * ldgf + n + c];
        gx[b * ldgx + c] += (pi / bnd) * d;
    }
}

int lanes_for(int n) {
    int w = 1;
    while (w < n && w < 64) w <<= 1;
    return w;
}

}  // namespace

extern "C" int64_t nfk_flows_bwd_workspace_bytes(int64_t batch, int32_t dim) {
    if (batch < 0 || dim <= 0) return 0;
    return (int64_t)ws_bytes(batch, dim);
}

extern "C" int nfk_planar_bwd(const float* x, int64_t ldx, const float* w, const float* u, const float* b,
                              const float* gz, int64_t ldgz, const float* glogdet, float* gx, int64_t ldgx,
                              float* gw, float* gu, float* gb, void* workspace, int64_t batch, int32_t dim,
                              int32_t nonlinearity, nfk_stream_t stream) {
    if (batch < 0 || dim <= 0 || dim > 16384) return nfk_set_error("nfk_planar_bwd: bad sizes");
    if (!x || !w || !u || !b || !gx || !gw || !gu || !gb || !workspace)
        return nfk_set_error("nfk_planar_bwd: null pointer");
    if (nonlinearity < 0 || nonlinearity > 2) return nfk_set_error("nfk_planar_bwd: bad nonlinearity");
    hipStream_t st = (hipStream_t)stream;
    Ws ws = ws_carve(workspace, batch, dim);
    if (batch > 0) {
        const int wl = lanes_for(dim);
        int64_t g = (batch + (4 * (64 / wl)) - 1) / (4 * (64 / wl));
        if (g > 65536) g = 65536;
        const size_t lds = (size_t)dim * sizeof(float);
#define CALL(W)                                                                                              \
    hipLaunchKernelGGL((k_planar_bwd_rows<W>), dim3((unsigned)g), dim3(256), lds, st, x, ldx, w, u, b, gz, ldgz, \
                       glogdet, gx, ldgx, ws.rows, batch, dim, nonlinearity);
        switch (wl) {
            case 1: CALL(1); break;
            case 2: CALL(2); break;
            case 4: CALL(4); break;
            case 8: CALL(8); break;
            case 16: CALL(16); break;
            case 32: CALL(32); break;
            default: CALL(64); break;
        }
#undef CALL
    }
    float* S = ws.sums;
    colsum(x, ldx, nullptr, 0, ws.rows, batch, dim, ws.part, S, st);                        // Gw
    if (gz != nullptr)
        colsum(gz, ldgz, nullptr, 0, ws.rows + batch, batch, dim, ws.part, S + dim, st);    // Gu
    else if (hipMemsetAsync(S + dim, 0, (size_t)dim * sizeof(float), st) != hipSuccess)
        return nfk_set_error("nfk_planar_bwd: memset failed");
    colsum(ws.rows, 1, nullptr, 0, nullptr, batch, 1, ws.part, S + 2 * dim, st);            // Gb
    colsum(ws.rows + 2 * batch, 1, nullptr, 0, nullptr, batch, 1, ws.part, S + 2 * dim + 1, st);  // C1
    hipLaunchKernelGGL(k_planar_bwd_params, dim3(1), dim3(256), 0, st, w, u, S, gw, gu, gb, dim, nonlinearity);
    return launch_status("nfk_planar_bwd");
}

extern "C" int nfk_actnorm_bwd(const float* x, int64_t ldx, const float* mu, const float* log_sigma, int32_t dim,
                               const float* gz, int64_t ldgz, const float* gld_scalar, float* gx, int64_t ldgx,
                               float* gmu, float* gls, void* workspace, int64_t batch, int32_t inverse,
                               nfk_stream_t stream) {
    if (batch < 0 || dim <= 0) return nfk_set_error("nfk_actnorm_bwd: bad sizes");
    if (!mu || !log_sigma || !gmu || !gls || !workspace) return nfk_set_error("nfk_actnorm_bwd: null pointer");
    if (batch > 0 && (!x || !gz || !gx)) return nfk_set_error("nfk_actnorm_bwd: null pointer");
    hipStream_t st = (hipStream_t)stream;
    Ws ws = ws_carve(workspace, batch, dim);
    if (batch > 0)
        hipLaunchKernelGGL(k_actnorm_bwd_x, dim3(grid_for(batch * (int64_t)dim, 256)), dim3(256), 0, st, gz, ldgz,
                           log_sigma, dim, gx, ldgx, batch, inverse);
    colsum(gz, ldgz, nullptr, 0, nullptr, batch, dim, ws.part, ws.sums, st);
    colsum(gz, ldgz, x, ldx, nullptr, batch, dim, ws.part, ws.sums + dim, st);
    hipLaunchKernelGGL(k_actnorm_bwd_params, dim3((unsigned)((dim + 255) / 256)), dim3(256), 0, st, mu, log_sigma,
                       ws.sums, gld_scalar, dim, gmu, gls, inverse);
    return launch_status("nfk_actnorm_bwd");
}

extern "C" int nfk_radial_bwd_scalars(const float* x, int64_t ldx, const float* x0, const float* log_alpha,
                                      const float* beta, const double* sumsq, const float* gz, int64_t ldgz,
                                      const float* gld_scalar, float* scal, void* workspace, int64_t batch,
                                      int32_t dim, nfk_stream_t stream) {
    if (batch < 0 || dim <= 0) return nfk_set_error("nfk_radial_bwd_scalars: bad sizes");
    if (!x0 || !log_alpha || !beta || !sumsq || !scal || !workspace)
        return nfk_set_error("nfk_radial_bwd_scalars: null pointer");
    if (batch > 0 && !x) return nfk_set_error("nfk_radial_bwd_scalars: null pointer");
    hipStream_t st = (hipStream_t)stream;
    Ws ws = ws_carve(workspace, batch, dim);
    float* S = ws.sums;
    if (gz != nullptr) {
        colsum(gz, ldgz, nullptr, 0, nullptr, batch, dim, ws.part, S, st);     // Gz
        colsum(gz, ldgz, x, ldx, nullptr, batch, dim, ws.part, S + dim, st);   // Gzx
    } else if (hipMemsetAsync(S, 0, 2 * (size_t)dim * sizeof(float), st) != hipSuccess) {
        return nfk_set_error("nfk_radial_bwd_scalars: memset failed");
    }
    colsum(x, ldx, nullptr, 0, nullptr, batch, dim, ws.part, S + 2 * dim, st);  // Xs
    hipLaunchKernelGGL(k_radial_bwd_scalars, dim3(1), dim3(256), 0, st, x0, log_alpha, beta, sumsq, S, gld_scalar,
                       dim, scal);
    return launch_status("nfk_radial_bwd_scalars");
}

extern "C" int nfk_radial_bwd_apply(const float* x, int64_t ldx, const float* x0, const float* gz, int64_t ldgz,
                                    const float* scal, float* gx, int64_t ldgx, float* gx0, void* workspace,
                                    int64_t batch, int32_t dim, nfk_stream_t stream) {
    if (batch < 0 || dim <= 0) return nfk_set_error("nfk_radial_bwd_apply: bad sizes");
    if (!x0 || !scal || !workspace) return nfk_set_error("nfk_radial_bwd_apply: null pointer");
    if (batch > 0 && (!x || !gx)) return nfk_set_error("nfk_radial_bwd_apply: null pointer");
    Ws ws = ws_carve(workspace, batch, dim);
    hipLaunchKernelGGL(k_radial_bwd_apply, dim3(grid_for(batch * (int64_t)dim, 256)), dim3(256), 0,
                       (hipStream_t)stream, x, ldx, x0, gz, ldgz, scal, ws.sums, gx, ldgx, gx0, batch, dim);
    return launch_status("nfk_radial_bwd_apply");
}

extern "C" int nfk_maf_bwd(const float* x, int64_t ldx, const float* init_param, const float* params, int64_t ldp,
                           const float* gout, int64_t ldgo, const float* glogdet, int32_t c0, int32_t c1, int32_t dim,
                           float* gx, int64_t ldgx, float* gparams, int64_t ldgp, float* ginit, void* workspace,
                           int64_t batch, int32_t inverse, nfk_stream_t stream) {
    if (batch < 0 || dim <= 0 || c0 < 0 || c1 > dim || c0 > c1) return nfk_set_error("nfk_maf_bwd: bad sizes");
    if (!init_param || !workspace) return nfk_set_error("nfk_maf_bwd: null pointer");
    if (batch > 0 && (!x || !gx)) return nfk_set_error("nfk_maf_bwd: null pointer");
    if (c1 > 1 && batch > 0 && (!params || !gparams)) return nfk_set_error("nfk_maf_bwd: null conditioner buffers");
    if (c0 == 0 && !ginit) return nfk_set_error("nfk_maf_bwd: null ginit");
    hipStream_t st = (hipStream_t)stream;
    Ws ws = ws_carve(workspace, batch, 2);
    if (batch > 0 && c0 < c1)
        hipLaunchKernelGGL(k_maf_bwd, dim3(grid_for(batch, 256)), dim3(256), 0, st, x, ldx, init_param, params, ldp,
                           gout, ldgo, glogdet, c0, c1, dim, gx, ldgx, gparams, ldgp, ws.rows, batch, inverse);
    if (c0 == 0) colsum(ws.rows, 2, nullptr, 0, nullptr, batch, 2, ws.part, ginit, st);
    return launch_status("nfk_maf_bwd");
}

extern "C" int nfk_trig_features_bwd(const float* x, int64_t ldx, const float* gfeat, int64_t ldgf, float* gx,
                                     int64_t ldgx, int64_t batch, int32_t n, double B, nfk_stream_t stream) {
    if (batch < 0 || n <= 0) return nfk_set_error("nfk_trig_features_bwd: bad sizes");
    if (batch == 0) return 0;
    if (!x || !gfeat || !gx) return nfk_set_error("nfk_trig_features_bwd: null pointer");
    int64_t g = (batch * n + 255) / 256;
    if (g > 16384) g = 16384;
    hipLaunchKernelGGL(k_trig_bwd, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, x, ldx, gfeat, ldgf, gx, ldgx,
                       batch, n, (float)M_PI, (float)B);
    return launch_status("nfk_trig_features_bwd");
}
