/*
 * nfk.h -- C ABI of libnfk.so, the MI355X (gfx950) kernels of the
 * normalizing-flow coupling-layer hot path.
 *
 * The reference (sherryli59/NormalizingFlow) is pure PyTorch and has no FFI:
 * each entry point below replaces a chain of ATen ops behind one of its Python
 * functions (file:line cited per function).  The Python host layer
 * (normalizingflow_amd/, re-exported as nf/) binds these with ctypes; see
 * INTEGRATION.md.
 *
 * Conventions
 *   - every pointer is device memory owned by the caller (the library never
 *     allocates or frees); fp32 unless the type says otherwise;
 *   - "ld*" arguments are row strides in ELEMENTS;
 *   - logdet_mode: 0 = do not touch logdet, 1 = logdet[b] = v, 2 = logdet[b] += v;
 *   - work is enqueued on `stream` (a hipStream_t); no call synchronises;
 *   - return value: 0 on success, a hipError_t (>0) from the launch, or
 *     NFK_EINVAL (<0) for bad arguments (nfk_last_error() says which).
 *   - data-dependent errors of the reference are recorded, not raised, as bits
 *     in *status (nullable) so the hot path never syncs; the host checks them
 *     lazily (see NFK_ST_*).
 */
#ifndef NFK_H_
#define NFK_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* nfk_stream_t; /* hipStream_t */

#define NFK_ABI_VERSION 2
#define NFK_EINVAL (-1)

/* status bits, OR-ed into *status by the kernels */
#define NFK_ST_INSIDE_SEEN 1 /* >=1 element inside [-B, B]; absent => the reference's
                                RuntimeError from torch.min of an empty tensor (utils.py:63) */
#define NFK_ST_NEG_DISC 2    /* negative discriminant in an inverse spline: the
                                reference's AssertionError (utils.py:121) */
#define NFK_ST_NAN_Z 4       /* a NaN in z reached the Normal prior: the reference's
                                ValueError from torch's MultivariateNormal argument
                                validation (prior.log_prob, nf/models.py:19) */

int nfk_abi_version(void);
const char* nfk_last_error(void);

/* ---------------------------------------------------------------------------
 * Rational-quadratic spline coupling.
 * Replaces NSF_CL.forward / NSF_CL.inverse minus the conditioner
 * (nf/flows.py:227-239, 241-253), unconstrained_RQS (nf/utils.py:27-56),
 * RQS (nf/utils.py:58-152) and searchsorted (nf/utils.py:20-25).
 *
 *   params     dense [batch, n_up, 3K-1]: per transformed element the
 *              (W[K], H[K], D[K-1]) block, i.e. psi(lower) reshaped as at
 *              flows.py:231, or cat(W, H, D) for the bare unconstrained_RQS.
 *   param_mode 0: raw NSF_CL conditioner output: W,H <- (right-left)*softmax,
 *                 D <- softplus (flows.py:233-235, where right-left = 2B)
 *                 before the spline's own normalisation;
 *              1: already the unconstrained_RQS arguments (utils.py:27);
 *              2: the bare RQS arguments (utils.py:58): params [batch, n_up, 3K+1]
 *                 with all K+1 derivative logits (no boundary constant).
 *   bounds     knots span [left, right] x [bottom, top] (utils.py:58-60)
 *   tails      1: identity outside [left, right] (unconstrained_RQS, which
 *                 passes left=bottom=-B, right=top=B); 0: every element is
 *                 splined (RQS; the caller checks the domain like utils.py:63)
 *   up_in[j]   column of x holding transformed element j; up_out[j] its column in z
 *   lo_in/lo_out: identity-copied ("lower") columns; n_lo may be 0.
 *   x and z must not alias.
 *   lad_out    nullable per-element log|det| [batch, n_up] with row stride ld_lad
 *   logdet     per-sample sum over j of log|det| (flows.py:238), per logdet_mode
 * ------------------------------------------------------------------------- */
int nfk_rqs_coupling(const float* x, int64_t ldx, const float* params,
                     const int32_t* up_in, const int32_t* up_out, int32_t n_up,
                     const int32_t* lo_in, const int32_t* lo_out, int32_t n_lo,
                     float* z, int64_t ldz, float* logdet, int32_t logdet_mode,
                     float* lad_out, int64_t ld_lad, int64_t batch, int32_t K,
                     double left, double right, double bottom, double top, int32_t tails,
                     double min_bin_width, double min_bin_height, double min_derivative,
                     int32_t param_mode, int32_t inverse, int32_t* status,
                     nfk_stream_t stream);

/* Backward (vector-Jacobian product) of nfk_rqs_coupling: same x / params /
 * maps / spline arguments as the forward call, plus the upstream gradients
 *   gz [batch, ldgz]   dL/dz (may be NULL: 0),  glogdet [batch] dL/dlog|det|
 *   (may be NULL: 0).
 * Writes gparams (dense, the layout of params) = dL/dparams, and
 *   gx[:, up_in[j]] = dL/dx_up,  gx[:, lo_in[q]] = gz[:, lo_out[q]]
 * (the conditioner's contribution to the lower coordinates is added by the
 * caller after its own backward).  No status words: the forward reported them.
 * Replaces the autograd graph of nf/flows.py:227-253 + nf/utils.py:27-152. */
int nfk_rqs_coupling_bwd(const float* x, int64_t ldx, const float* params,
                         const int32_t* up_in, const int32_t* up_out, int32_t n_up,
                         const int32_t* lo_in, const int32_t* lo_out, int32_t n_lo,
                         const float* gz, int64_t ldgz, const float* glogdet,
                         float* gparams, float* gx, int64_t ldgx, int64_t batch, int32_t K,
                         double left, double right, double bottom, double top, int32_t tails,
                         double min_bin_width, double min_bin_height, double min_derivative,
                         int32_t param_mode, int32_t inverse, nfk_stream_t stream);

/* MAF (nf/flows_1.py:159-195): per-coordinate affine map of the columns
 * [c0, c1) with (mu_i, alpha_i) = init_param[0..1] for i = 0 and
 * params[b*ldp + 2*(i - max(c0,1)) + {0,1}] (the conditioner outputs) otherwise.
 *   forward: out[b, dim-1-i] = (x[b,i] - mu_i) / exp(alpha_i),  log|det| -= alpha_i
 *   inverse: out[b, i] = mu_i + exp(alpha_i) * x[b, dim-1-i],   log|det| += alpha_i
 * (the output flip of flows_1.py:183 and the input flip of :187 are folded in).
 * The inverse is sequential in i: call it once per column after the
 * conditioner of that column has read out[:, :i]. */
int nfk_maf(const float* x, int64_t ldx, const float* init_param, const float* params,
            int64_t ldp, int32_t c0, int32_t c1, int32_t dim, float* out, int64_t ldo,
            float* logdet, int32_t logdet_mode, int64_t batch, int32_t inverse,
            nfk_stream_t stream);

/* ActNorm (nf/flows_1.py:198-215): z = x*exp(log_sigma) + mu (inverse
 * (z - mu)/exp(log_sigma)); log|det| = +-sum(log_sigma), a scalar, written to
 * ld_scalar (may be NULL) and/or written/accumulated into logdet[batch]. */
int nfk_actnorm(const float* x, int64_t ldx, const float* mu, const float* log_sigma,
                int32_t dim, float* z, int64_t ldz, float* logdet, int32_t logdet_mode,
                float* ld_scalar, int64_t batch, int32_t inverse, nfk_stream_t stream);

/* searchsorted (nf/utils.py:20-25), including its side effect:
 *   bin_locations[r, n_loc-1] += eps  (in place, fp32), then
 *   idx[r] = #{j : inputs[r] >= bin_locations[r, j]} - 1
 * bin_locations: dense [rows, n_loc]; inputs, idx: [rows]. */
int nfk_searchsorted(float* bin_locations, const float* inputs, int64_t* idx, int64_t rows,
                     int32_t n_loc, double eps, nfk_stream_t stream);

/* ---------------------------------------------------------------------------
 * Affine half-coupling of RealNVP (nf/flows.py:52-76):
 *   forward: out = t + in * exp(s),       logdet (+)= sum_j s
 *   inverse: out = (in - t) * exp(-s),    logdet (+)= sum_j (-s)
 * in/out may alias.  s and t share the row stride ld_st.
 * ------------------------------------------------------------------------- */
int nfk_affine_coupling(const float* x_in, int64_t ld_in, const float* s, const float* t,
                        int64_t ld_st, float* x_out, int64_t ld_out, float* logdet,
                        int32_t logdet_mode, int64_t batch, int32_t n, int32_t inverse,
                        nfk_stream_t stream);

/* Backward of nfk_affine_coupling (the VJP of flows.py:56/61 and 68/74 for
 * RealNVP's training path):
 *   forward  out = t + in e, e = exp(s):    g_in (+)= g e, g_t = g,    g_s = g in e + g_ld
 *   inverse  out = (in - t) e, e = exp(-s): g_in (+)= g e, g_t = -g e, g_s = -g out - g_ld
 * g = g_out (NULL: 0), g_ld = g_logdet[row] (NULL: 0); g_in written
 * (accumulate = 0) or added to (1); g_t may be NULL forward (it equals g_out).
 * g_s and g_t share the row stride ld_gst. */
int nfk_affine_coupling_bwd(const float* x_in, int64_t ld_in, const float* s, const float* t,
                            int64_t ld_st, const float* g_out, int64_t ld_g, const float* g_logdet,
                            float* g_in, int64_t ld_gin, int32_t accumulate, float* g_s, float* g_t,
                            int64_t ld_gst, int64_t batch, int32_t n, int32_t inverse,
                            nfk_stream_t stream);

/* ---------------------------------------------------------------------------
 * Planar flow forward (nf/flows_1.py:42-60), parameters w,u [dim], b [1].
 * nonlinearity: 0 tanh (u re-parameterised to u_hat), 1 leaky_relu, 2 elu
 * (u used as is; derivative exactly as flows_1.py:12-18, incl. its -0.01).
 * log|det| = log(|1 + phi.u_hat| + 1e-4).
 * ------------------------------------------------------------------------- */
int nfk_planar(const float* x, int64_t ldx, const float* w, const float* u, const float* b,
               float* z, int64_t ldz, float* logdet, int32_t logdet_mode, float* ld_out,
               int64_t batch, int32_t dim, int32_t nonlinearity, nfk_stream_t stream);

/* ---------------------------------------------------------------------------
 * Radial flow (nf/flows_1.py:85-97).  Its r = ||x - x0||_F is a BATCH-GLOBAL
 * norm, so the flow is two calls with an optional cross-rank all-reduce of
 * *sumsq in between:
 *   nfk_radial_sumsq: *sumsq = sum_{b,i} (x[b,i]-x0[i])^2 (fp64, deterministic;
 *                     workspace >= nfk_radial_workspace_elems() doubles)
 *   nfk_radial_apply: z = x + beta_hat*h*(x-x0); ld_scalar[0] = log|det|
 *                     (identical for every sample, shape [1] as in the reference)
 * ------------------------------------------------------------------------- */
int64_t nfk_radial_workspace_elems(void);
int nfk_radial_sumsq(const float* x, int64_t ldx, const float* x0, int64_t batch, int32_t dim,
                     double* workspace, double* sumsq, nfk_stream_t stream);
int nfk_radial_apply(const float* x, int64_t ldx, const float* x0, const float* log_alpha,
                     const float* beta, const double* sumsq, float* z, int64_t ldz,
                     float* ld_scalar, float* logdet, int32_t logdet_mode, int64_t batch,
                     int32_t dim, nfk_stream_t stream);

/* ---------------------------------------------------------------------------
 * Isotropic normal prior log-density epilogue: the reference's "Normal" prior
 * MultivariateNormal(0, var*I).log_prob (applications/src/setup.py:25-30)
 * combined with the flow log-det as in nf/models.py:34 and :39:
 *   out[b] = -0.5*(D*log(2pi) + sum_i (z_i/scale)^2) - half_log_det
 *            + sign * logdet[b]          (logdet nullable; sign = +1 or -1)
 * scale = the prior's Cholesky diagonal sqrt(var) (its scale_tril), and
 * half_log_det = sum_i log(scale) are passed in as torch evaluates them.
 *   status: nullable; NFK_ST_NAN_Z is OR-ed in when a row of z holds a NaN
 *           (torch validates the prior's argument: ValueError).
 * ------------------------------------------------------------------------- */
int nfk_normal_logprob(const float* z, int64_t ldz, const float* logdet, float* out,
                       int64_t batch, int32_t dim, float scale, float half_log_det,
                       int32_t sign, int32_t* status, nfk_stream_t stream);

/* ---------------------------------------------------------------------------
 * NSF_AR conditioner features (nf/flows.py:172-173, 183):
 *   feat[b, j] = cos(pi*x[b,j]/B), feat[b, n+j] = sin(pi*x[b,j]/B), j < n
 * ------------------------------------------------------------------------- */
int nfk_trig_features(const float* x, int64_t ldx, float* feat, int64_t ldf, int64_t batch,
                      int32_t n, double B, nfk_stream_t stream);

/* ---------------------------------------------------------------------------
 * Fused NSF_AR layer (nfk_fused_ar.hip): replaces NSF_AR.forward / inverse
 * (nf/flows.py:176-209) -- every coordinate's conditioner (FCNN(2i, 3K-1,
 * hidden) on the trig features of coordinates < i, flows.py:172-173, 183; the
 * init_param logits for coordinate 0) and its spline, ONE launch per layer.
 *   weights: a DEVICE array of (dim - 1) x 6 pointers, per conditioner
 *     i = 1 .. dim-1 in order {W1 [hidden][2i], b1, W2 [hidden][hidden], b2,
 *     W3 [3K-1][hidden], b3} (nn.Linear weight/bias, contiguous fp32);
 *   pack: nfk_fused_ar_pack_elems() floats, written by nfk_fused_ar_pack();
 *   x: the layer input [batch, dim] (forward: x, inverse: z); out: the output;
 *   logdet: mode 0 none, 1 write, 2 accumulate (the layer's sum over columns
 *     in column order); status: dim words (column i's reference errors: bit
 *     NFK_ST_INSIDE_SEEN when an element is inside [-B, B], NFK_ST_NEG_DISC).
 * Supported shapes: nfk_fused_ar_supported() != 0.
 * ------------------------------------------------------------------------- */
int nfk_fused_ar_supported(int32_t dim, int32_t hidden, int32_t K);
/* The inverse fused too (NSF_AR.inverse, flows.py:191-209)?  0 for the shapes
 * only the streamed forward covers (Polymer.yaml's 2048 coordinates): their
 * inverse runs per column. */
int nfk_fused_ar_inverse_supported(int32_t dim, int32_t hidden, int32_t K);
int64_t nfk_fused_ar_pack_elems(int32_t dim, int32_t hidden, int32_t K);
int nfk_fused_ar_pack(const float* const* weights, const float* init_param, int32_t dim, int32_t hidden,
                      int32_t K, float* pack, nfk_stream_t stream);
int nfk_fused_ar(const float* x, int64_t ldx, const float* pack, int32_t dim, int32_t hidden, int32_t K,
                 double tail_bound, float* out, int64_t ldo, float* logdet, int32_t logdet_mode,
                 int64_t batch, int32_t inverse, int32_t* status, nfk_stream_t stream);
/* The same with a workspace: a forward whose batch is too small to fill the
 * GPU splits the conditioners over workgroups (they are independent given x,
 * flows.py:182-189) when workspace holds nfk_fused_ar_workspace() floats (the
 * per-column log|det| terms, summed in column order: results bitwise those of
 * nfk_fused_ar).  A null or short workspace runs unsplit; 0 = none needed.
 * The shapes only the streamed forward covers (nfk_fused_ar_inverse_supported()
 * == 0) always need it: it also holds their trig operands. */
int64_t nfk_fused_ar_workspace(int32_t dim, int32_t hidden, int32_t K, int64_t batch, int32_t inverse);
int nfk_fused_ar_ws(const float* x, int64_t ldx, const float* pack, int32_t dim, int32_t hidden, int32_t K,
                    double tail_bound, float* out, int64_t ldo, float* logdet, int32_t logdet_mode,
                    int64_t batch, int32_t inverse, int32_t* status, float* workspace, int64_t workspace_floats,
                    nfk_stream_t stream);

/* ---------------------------------------------------------------------------
 * Fused NSF coupling layer: conditioner MLP (FCNN, flows.py:20-35) on MFMA
 * (fp16 two-way split with power-of-two pre-scaling, fp32 accumulation) +
 * spline epilogue, one launch per layer; the [batch, n_up, 3K-1] conditioner
 * output never touches HBM.  Replaces NSF_CL.forward/inverse (flows.py:227-253).
 *   wpack: weights re-packed by nfk_fused_nsf_pack() into MFMA fragment order
 *   (a device buffer of nfk_fused_nsf_pack_elems() floats).
 * Supported shapes: nfk_fused_nsf_supported() != 0.
 * ------------------------------------------------------------------------- */
int nfk_fused_nsf_supported(int32_t n_lo, int32_t n_up, int32_t hidden, int32_t K);
int64_t nfk_fused_nsf_pack_elems(int32_t n_lo, int32_t n_up, int32_t hidden, int32_t K);
int nfk_fused_nsf_pack(const float* w0, const float* b0, const float* w2, const float* b2,
                       const float* w4, const float* b4, int32_t n_lo, int32_t n_up,
                       int32_t hidden, int32_t K, float* wpack, nfk_stream_t stream);
int nfk_fused_nsf(const float* x, int64_t ldx, const float* wpack, const int32_t* up_in,
                  const int32_t* up_out, int32_t n_up, const int32_t* lo_in,
                  const int32_t* lo_out, int32_t n_lo, int32_t hidden, float* z, int64_t ldz,
                  float* logdet, int32_t logdet_mode, int64_t batch, int32_t K,
                  double tail_bound, int32_t inverse, int32_t* status, nfk_stream_t stream);
/* The same with a workspace of nfk_fused_nsf_workspace() floats: layers with a
 * conditioner wider than the instanced NSF_CL kernels (the applications'
 * H = 354, K = 32, setup.py:59-62) split their upper coordinates over
 * workgroups when the batch alone cannot fill the GPU, the per-coordinate
 * log|det| terms going through the workspace (summed in coordinate order:
 * bitwise the unsplit result).  0 floats = no split for this call. */
int64_t nfk_fused_nsf_workspace(int32_t n_lo, int32_t n_up, int32_t hidden, int32_t K, int64_t batch,
                                int32_t inverse);
int nfk_fused_nsf_ws(const float* x, int64_t ldx, const float* wpack, const int32_t* up_in,
                     const int32_t* up_out, int32_t n_up, const int32_t* lo_in, const int32_t* lo_out,
                     int32_t n_lo, int32_t hidden, float* z, int64_t ldz, float* logdet,
                     int32_t logdet_mode, int64_t batch, int32_t K, double tail_bound, int32_t inverse,
                     int32_t* status, float* workspace, int64_t workspace_floats, nfk_stream_t stream);

/* ---------------------------------------------------------------------------
 * Chain of fused NSF coupling layers in one launch: the layer loop of
 * NormalizingFlowModel.forward/inverse (nf/models.py:13-29) over nlayers
 * consecutive NSF_CL layers of one shape (n_lo, n_up, hidden, K, tail_bound)
 * and one direction.  Each wave keeps its 16 x rows in LDS from the first
 * layer to the last: HBM sees x once, z once and log|det| once per chain.
 * Results are bitwise those of nlayers nfk_fused_nsf launches (log|det| is
 * added layer by layer in the same order).
 *   wpacks: DEVICE array of nlayers pack pointers (nfk_fused_nsf_pack), in
 *           execution order.
 *   cmaps:  DEVICE int32 [nlayers * D + D], D = n_lo + n_up: for layer l,
 *           the tile columns of its lower inputs (n_lo) then of its upper
 *           inputs (n_up) -- the layer's lo_in/up_in composed with the column
 *           permutation of the layers before it (the tile keeps x's column
 *           order; a layer overwrites its upper columns in place) -- then, for
 *           every output column o of the last layer, the tile column holding it.
 *   status: nlayers words, one per layer (bits as nfk_rqs_coupling).
 *   log_prob: optional prior epilogue (NormalizingFlowModel.evaluate,
 *           models.py:37-40, Normal prior N(0, s^2 I), setup.py:25-30):
 *           log_prob[b] = log N(z_b; 0, prior_scale^2 I) + log|det|_b with
 *           prior_half_log_det = sum log(scale_tril diagonal) as torch has it
 *           (the constants of nfk_normal_logprob).  With log_prob given, z may
 *           be NULL (not written) and logdet NULL with logdet_mode 0; a NaN in
 *           z ORs NFK_ST_NAN_Z into status[0].
 * nlayers <= nfk_fused_nsf_chain_max() (0: shape not supported by the chain
 * form); x, z 16-byte aligned with ldx, ldz multiples of 4.
 * ------------------------------------------------------------------------- */
int nfk_fused_nsf_chain_max(int32_t n_lo, int32_t n_up, int32_t hidden, int32_t K);
int nfk_fused_nsf_chain(const float* x, int64_t ldx, const float* const* wpacks,
                        const int32_t* cmaps, int32_t nlayers, int32_t n_lo, int32_t n_up,
                        int32_t hidden, float* z, int64_t ldz, float* logdet,
                        int32_t logdet_mode, int64_t batch, int32_t K, double tail_bound,
                        int32_t inverse, int32_t* status, float* log_prob, float prior_scale,
                        float prior_half_log_det, nfk_stream_t stream);

/* ---------------------------------------------------------------------------
 * Training forward of a chain of fused NSF_CL layers (forward direction, the
 * two-tile chain's shapes: nfk_fused_nsf_chain_saved_ok != 0, nlayers >= 2):
 * nfk_fused_nsf_chain's z and log|det|, and in the same launch the INPUT of
 * every layer l >= 1 -- what that layer's backward needs (the per-layer
 * autograd node saves it, nf/models.py:13-20 run under autograd) -- written to
 * saves + (l - 1) * save_stride, rows of ld_saves floats, in that layer's own
 * column order (bitwise the z of layer l - 1).
 *   smaps: DEVICE int32 [(nlayers - 1) * D]: for layer l >= 1 and each of its
 *          input columns, the tile column holding it (the permutation the
 *          chain's cmaps compose at the start of layer l).
 * x, z, saves 16-byte aligned; ldx, ldz, ld_saves, save_stride multiples of 4;
 * D = n_lo + n_up a multiple of 4.
 * ------------------------------------------------------------------------- */
int nfk_fused_nsf_chain_saved_ok(int32_t n_lo, int32_t n_up, int32_t hidden, int32_t K, int32_t nlayers);
int nfk_fused_nsf_chain_saved(const float* x, int64_t ldx, const float* const* wpacks,
                              const int32_t* cmaps, int32_t nlayers, int32_t n_lo, int32_t n_up,
                              int32_t hidden, float* z, int64_t ldz, float* logdet,
                              int32_t logdet_mode, int64_t batch, int32_t K, double tail_bound,
                              int32_t* status, float* saves, int64_t ld_saves, int64_t save_stride,
                              const int32_t* smaps, nfk_stream_t stream);

/* ---------------------------------------------------------------------------
 * Training backward of one fused NSF_CL layer (the VJP of flows.py:227-253,
 * utils.py:58-152 at the layer input x): the conditioner recomputed on the
 * matrix cores as nfk_fused_nsf computes it, and the spline VJP of every
 * element on the logits in registers.  Writes
 *   gparams [batch, n_up, 3K-1]: dL/d(conditioner output), the input of the
 *            conditioner's own backward (GEMMs outside);
 *   gx [batch, D]: upper coordinates dL/dx through the spline, lower ones the
 *            identity part (gz of their output column; the conditioner's part
 *            is added by the caller);
 *   h1, h2 [batch, ldh]: the two tanh activations in columns [0, hidden) and
 *            1.0 at column hidden (ldh >= hidden + 1, a multiple of 4; rows
 *            16-byte aligned), for the weight-gradient GEMMs.
 * gz (dL/dz, [batch, D]) and glogdet (dL/dlog|det|, [batch]) are nullable.
 * vpack: nfk_fused_nsf_vjp_pack (the pack's records in 8-coordinate chunks and
 * their sub-record stream).  Supported: nfk_fused_nsf_vjp_pack_elems() > 0
 * (n_lo <= 32, D <= 128 and a multiple of 4; (KBH, tail, K) instantiated).
 * ------------------------------------------------------------------------- */
int64_t nfk_fused_nsf_vjp_pack_elems(int32_t n_lo, int32_t n_up, int32_t hidden, int32_t K);
int nfk_fused_nsf_vjp_pack(const float* w0, const float* b0, const float* w2, const float* b2,
                           const float* w4, const float* b4, int32_t n_lo, int32_t n_up,
                           int32_t hidden, int32_t K, float* vpack, nfk_stream_t stream);
int nfk_fused_nsf_vjp(const float* x, int64_t ldx, const float* vpack, const int32_t* up_in,
                      const int32_t* up_out, int32_t n_up, const int32_t* lo_in,
                      const int32_t* lo_out, int32_t n_lo, int32_t hidden, const float* gz,
                      int64_t ldgz, const float* glogdet, float* gparams, float* gx, int64_t ldgx,
                      float* h1, float* h2, int64_t ldh, int64_t batch, int32_t K,
                      double tail_bound, int32_t inverse, nfk_stream_t stream);

/* ---------------------------------------------------------------------------
 * Fused RealNVP layer: both affine half-couplings with their four FCNN
 * conditioners (s1, t1, s2, t2) in one launch; replaces RealNVP.forward /
 * inverse (flows.py:44-76).  x, z: [batch, 2*half_dim] row-major.
 *   nets: HOST array of 24 device pointers, nets s1, t1, s2, t2 in that order,
 *         each W0 [H, half_dim], b0, W2 [H, H], b2, W4 [half_dim, H], b4
 *         (nn.Linear weight/bias of network.0/.2/.4).
 * Supported shapes: nfk_fused_realnvp_supported() != 0 (half_dim = 16, 32,
 * 48 or 64; hidden <= 132).
 * ------------------------------------------------------------------------- */
int nfk_fused_realnvp_supported(int32_t half_dim, int32_t hidden);
int64_t nfk_fused_realnvp_pack_elems(int32_t half_dim, int32_t hidden);
int nfk_fused_realnvp_pack(const float* const* nets, int32_t half_dim, int32_t hidden, float* wpack,
                           nfk_stream_t stream);
int nfk_fused_realnvp(const float* x, int64_t ldx, const float* wpack, int32_t half_dim, int32_t hidden,
                      float* z, int64_t ldz, float* logdet, int32_t logdet_mode, int64_t batch,
                      int32_t inverse, nfk_stream_t stream);

/* ---------------------------------------------------------------------------
 * Chained RealNVP layers: nlayers consecutive RealNVP layers of one shape in
 * ONE launch (NormalizingFlowModel's layer loop, models.py:13-20 / 22-29 /
 * 37-40, over RealNVP.forward / inverse, flows.py:52-76).  Each layer's x is
 * the previous layer's z (the lower/upper halves keep their positions), so x
 * rows stay in LDS from the first layer to the last; z and log|det| are
 * bitwise those of nlayers nfk_fused_realnvp launches in the same order.
 *   wpacks: DEVICE array of nlayers pack pointers (nfk_fused_realnvp_pack:
 *           where nfk_fused_realnvp_chain_max() != 0 the pack also holds the
 *           chain's weight stream), in execution order (reversed layer order
 *           when inverse != 0, as the caller runs them).
 *   z: [batch, 2*half_dim] or NULL when log_prob is given.
 *   log_prob: nullable; the isotropic-Normal prior epilogue (the reference's
 *           "Normal" prior, applications/src/setup.py:25-30): log_prob[b] =
 *           log N(z_b; 0, prior_scale^2 I) + log|det|_b (prior_half_log_det =
 *           Sigma log of the scale_tril diagonal), and a NaN in z ORs
 *           NFK_ST_NAN_Z into status[0] (nullable).
 *   x, z rows 16-byte aligned (ldx, ldz multiples of 4).
 * nfk_fused_realnvp_chain_max(): most layers per launch (0: the chain form
 * does not apply to this shape; use nfk_fused_realnvp per layer).
 * ------------------------------------------------------------------------- */
int nfk_fused_realnvp_chain_max(int32_t half_dim, int32_t hidden);
int nfk_fused_realnvp_chain(const float* x, int64_t ldx, const float* const* wpacks, int32_t nlayers,
                            int32_t half_dim, int32_t hidden, float* z, int64_t ldz, float* logdet,
                            int32_t logdet_mode, int64_t batch, int32_t inverse, int32_t* status,
                            float* log_prob, float prior_scale, float prior_half_log_det,
                            nfk_stream_t stream);

/* ---------------------------------------------------------------------------
 * Training backward of the remaining flow classes (nfk_flows_bwd.hip): the
 * vector-Jacobian products autograd takes through flows_1.py's Planar
 * (:42-60), Radial (:85-97), ActNorm (:207-215), MAF (:171-195) and NSF_AR's
 * trig features (flows.py:172-173).  Batch sums (parameter gradients) are
 * deterministic (fixed-order fp64 column reductions, no atomics).
 *   workspace: device scratch of nfk_flows_bwd_workspace_bytes(batch, dim)
 *              bytes, 256-byte aligned (MAF: dim = 2).
 * Upstream gradients gz (dL/dz) and glogdet (dL/dlog|det|: [batch] per
 * sample, or a [1] scalar where the layer's log|det| is a scalar) are nullable.
 *
 * nfk_planar_bwd: gx [batch, dim]; gw, gu [dim], gb [1] (through the tanh
 *   re-parameterisation of u, flows_1.py:48-53).
 * nfk_actnorm_bwd: gx, gmu, gls (log|det| = +-sum(log_sigma): gld_scalar).
 * nfk_radial_bwd_scalars / _apply: two calls like the forward, because
 *   r = ||x - x0||_F is batch-global: scal[4] = [dL/dsumsq, dL/dlog_alpha,
 *   dL/dbeta, beta_hat h]; a sharded batch all-reduces (sums) scal[0] between
 *   the calls (the backward of the forward's all-reduce of sumsq); _apply
 *   writes gx and g_x0 [dim] (same workspace).
 * nfk_maf_bwd: columns [c0, c1) of nfk_maf with gout = dL/dout: gx at each
 *   column's input position (written), gparams (dL/d conditioner output, the
 *   layout of params), ginit [2] (= the batch sum, written when c0 == 0).
 *   The conditioners' own backward is the caller's (it adds into gx / gout).
 * nfk_trig_features_bwd: gx[:, :n] += dL/dx through nfk_trig_features.
 * ------------------------------------------------------------------------- */
int64_t nfk_flows_bwd_workspace_bytes(int64_t batch, int32_t dim);
int nfk_planar_bwd(const float* x, int64_t ldx, const float* w, const float* u, const float* b,
                   const float* gz, int64_t ldgz, const float* glogdet, float* gx, int64_t ldgx,
                   float* gw, float* gu, float* gb, void* workspace, int64_t batch, int32_t dim,
                   int32_t nonlinearity, nfk_stream_t stream);
int nfk_actnorm_bwd(const float* x, int64_t ldx, const float* mu, const float* log_sigma, int32_t dim,
                    const float* gz, int64_t ldgz, const float* gld_scalar, float* gx, int64_t ldgx,
                    float* gmu, float* gls, void* workspace, int64_t batch, int32_t inverse,
                    nfk_stream_t stream);
int nfk_radial_bwd_scalars(const float* x, int64_t ldx, const float* x0, const float* log_alpha,
                           const float* beta, const double* sumsq, const float* gz, int64_t ldgz,
                           const float* gld_scalar, float* scal, void* workspace, int64_t batch,
                           int32_t dim, nfk_stream_t stream);
int nfk_radial_bwd_apply(const float* x, int64_t ldx, const float* x0, const float* gz, int64_t ldgz,
                         const float* scal, float* gx, int64_t ldgx, float* gx0, void* workspace,
                         int64_t batch, int32_t dim, nfk_stream_t stream);
int nfk_maf_bwd(const float* x, int64_t ldx, const float* init_param, const float* params, int64_t ldp,
                const float* gout, int64_t ldgo, const float* glogdet, int32_t c0, int32_t c1,
                int32_t dim, float* gx, int64_t ldgx, float* gparams, int64_t ldgp, float* ginit,
                void* workspace, int64_t batch, int32_t inverse, nfk_stream_t stream);
int nfk_trig_features_bwd(const float* x, int64_t ldx, const float* gfeat, int64_t ldgf, float* gx,
                          int64_t ldgx, int64_t batch, int32_t n, double B, nfk_stream_t stream);

/* ---------------------------------------------------------------------------
 * Input-gradient GEMMs of the FCNN conditioner's backward (nfk_fcnn_bwd.hip;
 * the dX chain of flows.py:20-35 differentiated), tanh's backward fused:
 *   out[b, j] = (sum_p g[b, p] W[p, j]) * (1 - h[b, j]^2)    (h NULL: no factor)
 * W [P, H] row-major (an nn.Linear weight, out x in) re-packed once by
 * nfk_fcnn_dh_pack into nfk_fcnn_dh_pack_floats(P, H) floats (0: unsupported:
 * P a multiple of 4, H <= 128).  fp16 two-way split on the matrix cores, fp32
 * accumulation, per-row power-of-two scaling of g.  g rows 16-byte aligned.
 * out element (b, j) is out[b*ldo + j*out_col_stride]; accumulate != 0 adds
 * to it (e.g. the lower columns of a layer's dL/dx, written in place).
 * ------------------------------------------------------------------------- */
int64_t nfk_fcnn_dh_pack_floats(int32_t P, int32_t H);
/* [x[:, cols] | 1] for a weight gradient that carries its bias gradient in
 * the last column (the bias of flows.py:26's first nn.Linear):
 *   out[b, j] = x[b*ldx + cols[j]] (j < n), out[b, n] = 1, out[b, n+1 .. ldo) = 0
 * ldo a multiple of 4 and >= n + 1, out 16-byte aligned. */
int nfk_gather_cols_ones(const float* x, int64_t ldx, const int32_t* cols, int32_t n, int64_t batch,
                         float* out, int64_t ldo, nfk_stream_t stream);
int nfk_fcnn_dh_pack(const float* W, int32_t P, int32_t H, float* pack, nfk_stream_t stream);
int nfk_fcnn_dh(const float* g, int64_t ldg, int32_t P, const float* pack, const float* h, int64_t ldh,
                int32_t H, float* out, int64_t ldo, int64_t out_col_stride, int32_t accumulate,
                int64_t batch, nfk_stream_t stream);
/* The same kernel in forward form, for the training recompute of one FCNN
 * Linear (flows.py:26-31, nn.Linear + optional nn.Tanh):
 *   out[b, j] = act(sum_p x[b, p] W[p, j] + bias[j])   act = tanh if tanh_out
 * W [P, H] is the nn.Linear weight TRANSPOSED (in x out), packed by
 * nfk_fcnn_dh_pack; bias may be NULL.  x rows 16-byte aligned, out dense rows. */
int nfk_fcnn_linear(const float* x, int64_t ldx, int32_t P, const float* pack, const float* bias,
                    int32_t tanh_out, int32_t H, float* out, int64_t ldo, int64_t batch,
                    nfk_stream_t stream);

/* ---------------------------------------------------------------------------
 * RealNVP layers with wide conditioners at small batches (nfk_wide_rnvp.hip):
 * applications/input/Polymer_rnvp.yaml's RealNVP(2048, hidden 4000) at the
 * config's 40 rows and the driver's sample(100) (applications/examples/
 * polymer.py:29,37-41).  Replaces RealNVP.forward / inverse (nf/flows.py:52-76)
 * with its four FCNN conditioners (flows.py:20-35) when the layer is the
 * weight stream: every weight read once per layer.
 *
 * nfk_wlin_pack: an nn.Linear weight W [N, K] (out x in, row-major) re-packed
 * once into nfk_wlin_pack_floats(N, K) floats (fp16 hi/lo MFMA fragments of
 * 2^s W, one power of two per matrix).
 *
 * nfk_wide_rnvp: one RealNVP layer.  packs / biases: 12 device pointers each,
 * [6 c + 2 l + g] for half-coupling c (0: s1/t1, 1: s2/t2), Linear l (0, 1, 2
 * = network.0, .2, .4) and conditioner g (0 = s, 1 = t); biases are the
 * Linears' fp32 bias vectors.  x [batch, 2 half] (row stride ldx) -> z (ldz;
 * may equal x), logdet mode 0 none / 1 write / 2 accumulate (forward +sum s,
 * inverse -sum s, flows.py:61-62, 74-75).  workspace: at least
 * nfk_wide_rnvp_workspace(half, hidden, batch) floats, 16-byte aligned.  Rows
 * are processed 128 per pass (every pass streams the weights once).
 * half and hidden multiples of 4 (nfk_wide_rnvp_supported).
 * ------------------------------------------------------------------------- */
int64_t nfk_wlin_pack_floats(int32_t N, int32_t K);
int nfk_wlin_pack(const float* W, int32_t N, int32_t K, float* pack, nfk_stream_t stream);
int nfk_wide_rnvp_supported(int32_t half, int32_t hidden);
int64_t nfk_wide_rnvp_workspace(int32_t half, int32_t hidden, int64_t batch);
int nfk_wide_rnvp(const float* x, int64_t ldx, const float* const* packs, const float* const* biases, int32_t half,
                  int32_t hidden, float* z, int64_t ldz, float* logdet, int32_t logdet_mode, int64_t batch,
                  int32_t inverse, float* workspace, int64_t workspace_floats, nfk_stream_t stream);
/* nfk_wide_rnvp_chain: nlayers consecutive such layers in ONE call (the
 * model's layer loop, nf/models.py:13-29 / 22-35, over RealNVP layers of one
 * shape): packs / biases hold 12 pointers per layer in EXECUTION order (the
 * inverse's caller passes the layers last to first).  Bitwise the per-layer
 * calls; the last half-coupling of each layer also writes the next layer's
 * input fragments, so only the first layer converts x.  workspace:
 * nfk_wide_rnvp_chain_workspace(half, hidden, batch) floats. */
int64_t nfk_wide_rnvp_chain_workspace(int32_t half, int32_t hidden, int64_t batch);
int nfk_wide_rnvp_chain(const float* x, int64_t ldx, const float* const* packs, const float* const* biases,
                        int32_t nlayers, int32_t half, int32_t hidden, float* z, int64_t ldz, float* logdet,
                        int32_t logdet_mode, int64_t batch, int32_t inverse, float* workspace,
                        int64_t workspace_floats, nfk_stream_t stream);

/* ---------------------------------------------------------------------------
 * NSF_AR inverse for the layers the fused kernel's inverse does not take
 * (nfk_fused_ar_inverse_supported == 0: Polymer.yaml's 2,048 coordinates),
 * nfk_ar_seqinv.hip: NSF_AR.inverse (nf/flows.py:193-209) column by column,
 * one launch per coordinate issued from the library (per row, one workgroup
 * finishes conditioner i: its layer-1 partial sums plus x_{i-1}'s two
 * features, layers 2-3, the spline's inverse and the trig features of x_i;
 * beside them, workgroups run conditioner i+1's layer 1 over the features
 * already known, 64 at a time), fp32 arithmetic, the weights read in
 * place.  weights: a HOST array of 6 (dim - 1) device pointers (W1, b1, W2,
 * b2, W3, b3 of conditioners 1 .. dim-1, fp32 contiguous nn.Linear tensors: the
 * entries of the table nfk_fused_ar_pack reads; each launch takes its
 * conditioners' pointers as arguments); init_param [3K-1].  z -> x [batch, dim],
 * logdet mode 0/1/2 (the inverse's -log|det|), status [dim] (nullable).
 * workspace: nfk_ar_seqinv_workspace(dim, hidden, K, batch) floats.  64 rows
 * per pass.  hidden <= 128, K in {4, 8, 10, 16, 32}.
 * ------------------------------------------------------------------------- */
int nfk_ar_seqinv_supported(int32_t dim, int32_t hidden, int32_t K);
int64_t nfk_ar_seqinv_workspace(int32_t dim, int32_t hidden, int32_t K, int64_t batch);
int nfk_ar_seqinv(const float* z, int64_t ldz, const float* const* weights, const float* init_param, int32_t dim,
                  int32_t hidden, int32_t K, double tail_bound, float* x, int64_t ldx, float* logdet,
                  int32_t logdet_mode, int64_t batch, int32_t* status, float* workspace, int64_t workspace_floats,
                  nfk_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* NFK_H_ */
