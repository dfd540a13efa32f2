"""fp32-accurate GEMMs on the fp16 matrix cores, for the training path.

The NSF_CL backward (flows.NSF_CL._vjp) recomputes the conditioner FCNN
(nf/flows.py:20-35: Linear -> Tanh -> Linear -> Tanh -> Linear) and
differentiates it; in fp32 those GEMMs run at the fp32 matrix rate (157 TF
dense on MI355X, ~43 TF achieved by hipBLASLt on these skinny shapes).  Here
every product A.B runs as the two-way fp16 split the fused forward kernel
uses (nfk_fused_impl.h): A = 2^-a (Ah + Al), B = 2^-b (Bh + Bl) with
power-of-two per-tensor scales that put max|A|, max|B| just under 2^15, and

    A.B ~= 2^-(a+b) (Al.Bh + Ah.Bl + Ah.Bh)

as three fp16 GEMMs with fp32 accumulation and fp32 output
(torch.mm(..., out_dtype=torch.float32), hipBLASLt).  The dropped Al.Bl term
is 2^-22 relative; the products of fp16 values are exact in fp32.  Scales are
device tensors (no host sync).  Used only where autograd needs gradients;
inference runs the fused kernels.
"""
from __future__ import annotations

import torch

F16 = torch.float16
F32 = torch.float32


def _split(t):
    """(hi, lo, unscale): t = unscale * (hi + lo) to ~2^-22 relative."""
    m = t.abs().amax()
    e = torch.frexp(m).exponent            # m < 2^e (m = 0: e = 0)
    s = torch.ldexp(torch.ones((), dtype=F32, device=t.device), 15 - e.clamp(-100, 100))
    ts = t * s
    hi = ts.to(F16)
    lo = (ts - hi.to(F32)).to(F16)
    return hi, lo, 1.0 / s


def mm3(a, b):
    """a [m, k] @ b [k, n] in fp32 precision from three fp16 GEMMs."""
    ah, al, ua = _split(a)
    bh, bl, ub = _split(b)
    c = torch.mm(al, bh, out_dtype=F32)
    c = c + torch.mm(ah, bl, out_dtype=F32)
    c = c + torch.mm(ah, bh, out_dtype=F32)
    return c * (ua * ub)


class _SplitLinear(torch.autograd.Function):
    """y = x W^T + b (nn.Linear) with mm3 products, forward and backward."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        y = mm3(x, w.t())
        return y + b if b is not None else y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx = mm3(gy, w) if ctx.needs_input_grad[0] else None
        gw = mm3(gy.t(), x) if ctx.needs_input_grad[1] else None
        gb = gy.sum(0) if ctx.has_b and ctx.needs_input_grad[2] else None
        return gx, gw, gb


def linear(x, w, b=None):
    return _SplitLinear.apply(x, w, b)


def fcnn(p, prefix, x):
    """The stock FCNN (flows.py:20-35) with parameters p[prefix + "network.{0,2,4}.*"]."""
    g = lambda i, n: p.get("%snetwork.%d.%s" % (prefix, i, n))
    h = torch.tanh(linear(x, g(0, "weight"), g(0, "bias")))
    h = torch.tanh(linear(h, g(2, "weight"), g(2, "bias")))
    return linear(h, g(4, "weight"), g(4, "bias"))
