"""Recompute-backward of the stock FCNN conditioner (nf/flows.py:20-35:
Linear -> Tanh -> Linear -> Tanh -> Linear) for the training path.

The layer kernels save only their input; the backward recomputes the three
activations and forms the vector-Jacobian products by hand instead of through
autograd, so each product is a GEMM of the shape that suits the device:

* input and hidden gradients (g @ W, M = batch, tanh's backward fused):
  nfk_fcnn_dh on the matrix cores (dh), else one library GEMM each;
* weight gradients g^T h reduce over the batch (against [h | 1] when the
  activations come with a ones column, as nfk_fused_nsf_vjp writes them, so
  the same GEMM's last column is the bias gradient; else a GEMM and a column
  sum) (K = 2^20 rows against 100 x 100 or 736 x 100 outputs).  A single GEMM of that shape has a few dozen output
  tiles for 256 CUs, so the batch is split into S slices and the S partial
  products (one batched GEMM) summed: split-K by hand (wgrad).

Same values as autograd through nn.Linear / nn.Tanh up to fp32 summation
order (tests/test_gpu_grad.py checks the layer gradients against the oracle's
autograd)."""
from __future__ import annotations

import torch

from . import config
from . import kernels as K_

_WG_ROWS = 8192   # rows per split-K slice of the weight-gradient GEMMs
_WG_SLICES = 64   # at most this many slices


def linears(p, pre):
    """(W1, b1, W2, b2, W3, b3) of FCNN ``pre`` from the name -> tensor map."""
    return tuple(p[pre + "network.%d.%s" % (i, k)] for i in (0, 2, 4) for k in ("weight", "bias"))


def forward_saved(p, pre, x):
    """psi(x) and the activations its backward needs: (x, h1, h2), dense [B, H]."""
    W1, b1, W2, b2, W3, b3 = linears(p, pre)
    if config.USE_FCNN_FWD and _kernel_ok(x) and all(K_.fcnn_dh_pack_floats(W.shape[1], W.shape[0]) > 0
                                                     for W in (W1, W2, W3)):
        # nfk_fcnn_linear: bias and tanh in the GEMM's epilogue
        def lin(a, W, b, act):
            out = torch.empty(a.shape[0], W.shape[0], dtype=a.dtype, device=a.device)
            K_.fcnn_linear(a, K_.fcnn_dh_pack(W.t()), (W.shape[1], W.shape[0]), b.contiguous(), out, tanh=act)
            return out
        h1 = lin(x, W1, b1, True)
        h2 = lin(h1, W2, b2, True)
        return lin(h2, W3, b3, False), (x, h1, h2)
    # W^T materialised: with the transposed view hipBLASLt picked a kernel 2.1x
    # slower for the 100 x 100 layer at 2^20 rows (tools/ubench_linear2.py)
    h1 = torch.tanh(torch.addmm(b1, x, W1.t().contiguous()))
    h2 = torch.tanh(torch.addmm(b2, h1, W2.t().contiguous()))
    return torch.addmm(b3, h2, W3.t().contiguous()), (x, h1, h2)


def wgrad(g, h):
    """g^T h for g [B, M], h [B, N]: split-K fp32 library GEMMs over batch
    slices (see module doc), summed in slice order."""
    B = g.shape[0]
    S = min(_WG_SLICES, B // _WG_ROWS)
    if S <= 1:
        return g.t() @ h
    R = B // S
    # (h^T g)^T: the batched GEMM with the narrow operand first measured 3 %
    # faster than g^T h at c3's [736 x 101] (tools/ubench_wgrad.py)
    out = torch.bmm(h[:S * R].view(S, R, -1).transpose(1, 2), g[:S * R].view(S, R, -1)).sum(0).t()
    if S * R < B:
        out += g[S * R:].t() @ h[S * R:]
    return out


def _kernel_ok(a):
    """a can feed nfk_fcnn_dh / nfk_fcnn_linear: HIP fp32, unit column
    stride, rows 16-byte aligned (a row-strided view such as x's lower half is
    fine)."""
    return a.is_cuda and a.dtype == torch.float32 and a.dim() == 2 and a.shape[0] > 0 \
        and (a.shape[1] == 1 or a.stride(1) == 1) and a.stride(0) % 4 == 0 and a.data_ptr() % 16 == 0


def dh(g, W, h, into=None):
    """(g @ W) * (1 - h^2) (h None: g @ W): nfk_fcnn_dh on the matrix cores
    where the shape allows (config.USE_FCNN_DH), else a library GEMM.  With
    ``into`` (a [B, H] view, any column stride) the result is added to it in
    place and None is returned."""
    if config.USE_FCNN_DH and _kernel_ok(g) and K_.fcnn_dh_pack_floats(*W.shape) > 0:
        # packed at every call: in training the weights change every step, and
        # a cache keyed on storage pointers can be fooled by a freed weight's
        # address coming back
        pk = K_.fcnn_dh_pack(W)
        if pk is not None:
            if into is not None:
                K_.fcnn_dh(g, pk, tuple(W.shape), h, into, accumulate=True)
                return None
            out = torch.empty(g.shape[0], W.shape[1], dtype=g.dtype, device=g.device)
            K_.fcnn_dh(g, pk, tuple(W.shape), h, out)
            return out
    y = g @ W
    y = y if h is None else torch.ops.aten.tanh_backward(y, h)
    if into is not None:
        into += y
        return None
    return y


def vjp(p, pre, cache, g, need_x, need, gx_into=None):
    """(dL/dx or None, {name: grad}) of psi at the cached activations for the
    output gradient g; ``need``: the parameter names whose gradient is wanted.
    With ``gx_into`` (a view of the caller's dL/dx, e.g. the lower columns),
    dL/dx is added into it and None returned in its place."""
    x, h1a, h2a = cache
    W1, b1, W2, b2, W3, b3 = linears(p, pre)
    H = W1.shape[0]
    # the activations come as [B, H] or, from nfk_fused_nsf_vjp, as [h | 1];
    # the input likewise as x or [x | 1] (kernels.gather_cols_ones)
    h1, h2 = h1a[:, :H], h2a[:, :H]
    names = [pre + "network.%d.%s" % (i, k) for i in (0, 2, 4) for k in ("weight", "bias")]
    grads = {}

    def put(i, g_out, act_a, n_in):
        """weight and bias gradient of Linear i: one GEMM against [act | 1] (its
        last column the bias gradient), or a GEMM and a column sum"""
        nw, nb = names[2 * i], names[2 * i + 1]
        if nw in need or nb in need:
            if act_a.shape[1] == n_in + 1:
                wb = wgrad(g_out, act_a)
                if nw in need:
                    grads[nw] = wb[:, :-1].contiguous()
                if nb in need:
                    grads[nb] = wb[:, -1].contiguous()
            else:
                if nw in need:
                    grads[nw] = wgrad(g_out, act_a).contiguous()
                if nb in need:
                    grads[nb] = g_out.sum(0)

    put(2, g, h2a, H)
    ga2 = dh(g, W3, h2)
    put(1, ga2, h1a, H)
    ga1 = dh(ga2, W2, h1)
    put(0, ga1, x, W1.shape[1])
    gx = dh(ga1, W1, None, into=gx_into) if need_x else None
    return gx, grads
