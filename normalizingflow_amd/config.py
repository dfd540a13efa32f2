"""Runtime switches of the host layer (plain module globals).

STRICT_CHECKS  raise the reference's data-dependent errors (RuntimeError when a
               spline layer has no element inside [-B, B], AssertionError on a
               negative discriminant) after each top-level call.  Costs one
               device->host read of the status words per call; the kernels
               themselves never sync.
USE_FUSED      run NSF_CL layers whose conditioner is the stock FCNN through the
               fused MFMA kernel (nfk_fused_nsf) when the shape is supported;
               otherwise conditioner GEMMs + the streaming spline kernel.
USE_CHAIN      in inference, run consecutive fused NSF_CL layers of one shape as
               one nfk_fused_nsf_chain launch (x resident in LDS across the
               layers); results are bitwise those of the per-layer launches.
SPLIT_GEMM     training: the NSF_CL conditioner's recompute-backward GEMMs as
               fp16-split products on the fp16 matrix cores (split_gemm.py,
               fp32-accurate) instead of fp32 GEMMs.  Off: torch.mm with
               out_dtype=float32 measured 3.5x slower than the fp32 GEMMs
               (c3 train step 468 vs 135 ms at 2^20).
"""
STRICT_CHECKS = True
USE_FUSED = True
USE_CHAIN = True
SPLIT_GEMM = False
