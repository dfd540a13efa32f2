"""Runtime switches of the host layer (plain module globals).

STRICT_CHECKS  raise the reference's data-dependent errors (RuntimeError when a
               spline layer has no element inside [-B, B], AssertionError on a
               negative discriminant, ValueError when a NaN z reaches a
               validating Normal prior) from the kernels' status words.
               True: after each top-level call (one device->host read, which
               waits for the call's kernels).  "deferred": the words are copied
               to pinned memory without a sync and their errors raised at a
               later call once they have landed, or by
               flows.flush_status_checks() -- the device queue never drains for
               a check (bench.py's mode).  False: never checked.
USE_FUSED      run NSF_CL layers whose conditioner is the stock FCNN through the
               fused MFMA kernel (nfk_fused_nsf) when the shape is supported;
               otherwise conditioner GEMMs + the streaming spline kernel.
USE_CHAIN      in inference, run consecutive fused NSF_CL layers of one shape as
               one nfk_fused_nsf_chain launch (x resident in LDS across the
               layers); results are bitwise those of the per-layer launches.
USE_TRAIN_CHAIN training (forward direction under autograd): consecutive fused
               NSF_CL layers of a two-tile-chain shape run as ONE
               nfk_fused_nsf_chain_saved launch that also writes each layer's
               input for its backward (models._ChainFn); off: one autograd
               node and one launch per layer.  Values and gradients are bitwise
               those of the per-layer path.
USE_FUSED_VJP  training: NSF_CL's backward through nfk_fused_nsf_vjp (conditioner
               recompute on the matrix cores + spline VJP in one kernel) where
               the shape is supported; off: recompute GEMMs + nfk_rqs_coupling_bwd.
FUSED_VJP_MAX_ROWS  training: the largest batch the fused VJP kernel takes (None:
               any); larger batches run the unfused backward (recompute GEMMs +
               nfk_rqs_coupling_bwd).  A switch, not a correctness gate: the fused
               VJP is bitwise reproducible at every batch.
USE_FCNN_DH    training: the stock FCNN backward's input-gradient GEMMs (g W,
               tanh's backward fused) on nfk_fcnn_dh (fp16-split MFMA) where
               the shape is supported; off: fp32 library GEMMs + tanh_backward.
USE_FCNN_FWD   training: the stock FCNN's recompute forward (Linear + bias +
               Tanh) on nfk_fcnn_linear, the same kernel in forward form;
               off: library GEMMs (addmm) + tanh.
AR_BATCHED_VJP_BYTES  training: NSF_AR's forward-direction backward recomputes and
               differentiates ALL its conditioners at once (batched GEMMs over
               the dim - 1 conditioners, one spline-VJP launch for every column)
               when its activations take at most this many bytes; above it,
               one column at a time.  0: always per column.
AR_WORKSPACE_BYTES  the streamed NSF_AR forward (shapes like Polymer.yaml's 2,048
               coordinates) needs a workspace of ~24 KB per row (per-column
               log|det| terms and the trig operands); a batch whose workspace
               would exceed this many bytes runs as several launches over
               row blocks (results bitwise the same: rows are independent).
USE_WIDE_RNVP  RealNVP layers whose conditioners are too wide for the fused kernel
               (Polymer_rnvp.yaml: hidden 4000) run as a weight stream
               (nfk_wide_rnvp: every Linear packed once, each weight read once
               per layer) at batches of at most WIDE_RNVP_MAX_ROWS rows (128 per
               pass); larger batches, or off: library GEMMs + the affine kernel.
USE_AR_SEQINV  the NSF_AR inverse of layers the fused inverse does not take (Polymer's
               2,048 coordinates) through nfk_ar_seqinv (two launches per column
               issued by the library, fp32); off: the per-column host loop.
"""
STRICT_CHECKS = True
USE_FUSED = True
USE_CHAIN = True
USE_TRAIN_CHAIN = True
USE_FUSED_VJP = True
FUSED_VJP_MAX_ROWS = None
USE_FCNN_DH = True
USE_FCNN_FWD = True
AR_BATCHED_VJP_BYTES = 4 << 30
AR_WORKSPACE_BYTES = 1 << 30
USE_WIDE_RNVP = True
WIDE_RNVP_MAX_ROWS = 1024
USE_AR_SEQINV = True
