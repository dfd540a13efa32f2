"""Differentiable torch restatement of the flow layers, for gradients.

The HIP kernels compute forward/inverse; when autograd needs gradients,
``normalizingflow_amd.autograd`` recomputes a layer with these functions on
the same device and back-propagates through them (until backward
kernels land, training uses a restated torch path).  They follow the reference
math (nf/utils.py:20-152, nf/flows.py:20-253, nf/flows_1.py:21-97) in a form
suited to the GPU: the spline tails use ``torch.where`` on clamped inputs
instead of boolean compaction (no host syncs, and no NaN gradients from the
unused branch), and nothing is written in place.  Values agree with the
reference to fp32 rounding; gradients are those of the same functions.

Parameters are passed as a dict name -> tensor (the layer's own
``named_parameters`` keys), so the recomputation can differentiate with
respect to detached copies; conditioners run through
``torch.func.functional_call`` so any ``base_network`` works.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

MIN_BIN_WIDTH = 1e-3
MIN_BIN_HEIGHT = 1e-3
MIN_DERIVATIVE = 1e-3


def conditioner(layer, p, name, x):
    """Run the layer's sub-network ``name`` (an FCNN, flows.py:20-35, or any
    user ``base_network``) on x with the parameters taken from ``p``."""
    mod = layer.get_submodule(name)
    pre = name + "."
    sub = {k[len(pre):]: v for k, v in p.items() if k.startswith(pre)}
    return torch.func.functional_call(mod, sub, (x,))


def _knots(u, lo, hi, min_bin):
    """softmax -> floor -> cumsum -> pinned ends (utils.py:73-80 / 84-91)."""
    k = u.shape[-1]
    w = min_bin + (1 - min_bin * k) * torch.softmax(u, dim=-1)
    c = F.pad(torch.cumsum(w, dim=-1), (1, 0), value=0.0) * (hi - lo) + lo
    c = torch.cat([torch.full_like(c[..., :1], lo), c[..., 1:-1], torch.full_like(c[..., :1], hi)], dim=-1)
    return c, c[..., 1:] - c[..., :-1]


def rq_spline(x, uw, uh, ud, inverse, lo, hi):
    """RQS (utils.py:58-152) for inputs inside [lo, hi]; ud holds all K+1
    derivative logits.  Returns (out, logabsdet)."""
    cw, w = _knots(uw, lo, hi, MIN_BIN_WIDTH)
    ch, h = _knots(uh, lo, hi, MIN_BIN_HEIGHT)
    d = MIN_DERIVATIVE + F.softplus(ud)
    edges = (ch if inverse else cw).detach().clone()
    edges[..., -1] += 1e-6  # searchsorted's eps (utils.py:20-25)
    k = (torch.sum(x[..., None] >= edges, dim=-1) - 1).clamp(0, w.shape[-1] - 1)[..., None]
    g = lambda t: t.gather(-1, k)[..., 0]
    cw_k, w_k, ch_k, h_k = g(cw), g(w), g(ch), g(h)
    delta = h / w
    dl_k, d_k, d_k1 = g(delta), g(d), g(d[..., 1:])
    gap = d_k + d_k1 - 2 * dl_k
    if inverse:
        y = x - ch_k
        a = y * gap + h_k * (dl_k - d_k)
        b = h_k * d_k - y * gap
        c = -dl_k * y
        disc = (b.pow(2) - 4 * a * c).clamp_min(0.0)
        th = (2 * c) / (-b - torch.sqrt(disc))
        out = th * w_k + cw_k
    else:
        th = (x - cw_k) / w_k
    t1mt = th * (1 - th)
    den = dl_k + gap * t1mt
    if not inverse:
        out = ch_k + h_k * (dl_k * th.pow(2) + d_k * t1mt) / den
    dnum = dl_k.pow(2) * (d_k1 * th.pow(2) + 2 * dl_k * t1mt + d_k * (1 - th).pow(2))
    lad = torch.log(dnum) - 2 * torch.log(den)
    return out, (-lad if inverse else lad)


def unconstrained_rq_spline(x, uw, uh, ud, inverse, tail_bound):
    """unconstrained_RQS (utils.py:27-56): identity outside [-B, B]; the two
    boundary derivative logits are the constant of utils.py:37."""
    const = float(np.log(np.exp(1 - MIN_DERIVATIVE) - 1))
    pad = torch.full_like(ud[..., :1], const)
    udp = torch.cat([pad, ud, pad], dim=-1)
    inside = (x >= -tail_bound) & (x <= tail_bound)
    xs = torch.where(inside, x, torch.zeros_like(x))
    out, lad = rq_spline(xs, uw, uh, udp, inverse, -tail_bound, tail_bound)
    return torch.where(inside, out, x), torch.where(inside, lad, torch.zeros_like(lad))


def _nsf_params(out, K, B):
    W, H, D = torch.split(out, K, dim=-1)
    return 2 * B * torch.softmax(W, dim=-1), 2 * B * torch.softmax(H, dim=-1), F.softplus(D)


def nsf_cl(layer, x, p, inverse):
    """NSF_CL.forward / inverse (flows.py:227-253)."""
    size, dim, K, B = layer.size, layer.dim, layer.K, layer.B
    mask = [int(m) for m in layer.mask]
    unm = [int(m) for m in layer.unmasked]
    xv = x.reshape(-1, size, dim)
    lower = xv[:, :, mask].flatten(1)
    upper = xv[:, :, unm].flatten(1)
    out = conditioner(layer, p, "psi", lower).reshape(-1, len(unm) * size, 3 * K - 1)
    W, H, D = _nsf_params(out, K, B)
    up2, lad = unconstrained_rq_spline(upper, W, H, D, inverse, float(B))
    z = torch.cat([lower.reshape(-1, size, len(mask)), up2.reshape(-1, size, len(unm))], dim=2).flatten(1)
    return z, lad.sum(dim=1)


def realnvp(layer, x, p, inverse):
    """RealNVP.forward / inverse (flows.py:52-76)."""
    h = layer.dim // 2
    lo, up = x[:, :h], x[:, h:]
    if not inverse:
        s1 = conditioner(layer, p, "s1", lo)
        up = conditioner(layer, p, "t1", lo) + up * torch.exp(s1)
        s2 = conditioner(layer, p, "s2", up)
        lo = conditioner(layer, p, "t2", up) + lo * torch.exp(s2)
        return torch.cat([lo, up], dim=1), s1.sum(dim=1) + s2.sum(dim=1)
    s2 = conditioner(layer, p, "s2", up)
    lo = (lo - conditioner(layer, p, "t2", up)) * torch.exp(-s2)
    s1 = conditioner(layer, p, "s1", lo)
    up = (up - conditioner(layer, p, "t1", lo)) * torch.exp(-s1)
    return torch.cat([lo, up], dim=1), (-s1).sum(dim=1) + (-s2).sum(dim=1)


def nsf_ar(layer, x, p, inverse):
    """NSF_AR.forward / inverse (flows.py:174-209): dimension i is conditioned
    on trig features of the first i coordinates of the input (forward) or of
    the output built so far (inverse)."""
    dim, K, B = layer.dim, layer.K, layer.B
    cols, ld = [], torch.zeros(x.shape[0], dtype=x.dtype, device=x.device)
    for i in range(dim):
        if i == 0:
            out = p["init_param"].expand(x.shape[0], 3 * K - 1)
        else:
            src = torch.stack(cols, dim=1) if inverse else x[:, :i]
            feat = torch.cat([torch.cos(math.pi * src / B), torch.sin(math.pi * src / B)], dim=-1)
            out = conditioner(layer, p, "layers.%d" % (i - 1), feat)
        W, H, D = _nsf_params(out, K, B)
        zi, l = unconstrained_rq_spline(x[:, i], W, H, D, inverse, float(B))
        cols.append(zi)
        ld = ld + l
    return torch.stack(cols, dim=1), ld


def planar(layer, x, p, inverse):
    """Planar.forward (flows_1.py:42-60); the activation derivative is taken
    on the input's device (the reference builds it as a CPU FloatTensor)."""
    if inverse:
        raise NotImplementedError("Planar flow has no algebraic inverse.")
    w, u, b = p["w"], p["u"], p["b"]
    act = layer.h
    if act is torch.tanh:
        wu = w @ u
        u = u + (torch.log(1 + torch.exp(wu)) - wu - 1) * w / torch.norm(w) ** 2
    lin = (x @ w)[:, None] + b
    z = x + u * act(lin)
    if act is torch.tanh:
        dh = 1 - torch.tanh(lin) ** 2
    elif act is F.leaky_relu:
        dh = (lin > 0).to(x.dtype) + (lin < 0).to(x.dtype) * -0.01
    else:
        dh = (lin > 0).to(x.dtype) + (lin < 0).to(x.dtype) * torch.exp(lin)
    phi = dh * w
    return z, torch.log(torch.abs(1 + phi @ u) + 1e-4)


def radial(layer, x, p, inverse):
    """Radial.forward (flows_1.py:85-97): r is the norm over the whole batch
    (all ranks' shards when the layer has a process group)."""
    if inverse:
        raise AttributeError("'Radial' object has no attribute 'inverse'")
    x0, la, be = p["x0"], p["log_alpha"], p["beta"]
    n = x.shape[1]
    sq = torch.sum((x - x0) ** 2)
    if getattr(layer, "process_group", None) is not None:
        import torch.distributed.nn.functional as dnn
        sq = dnn.all_reduce(sq, group=layer.process_group)
    r = torch.sqrt(sq)
    ea = torch.exp(la)
    h = 1 / (ea + r)
    bh = -ea + torch.log(1 + torch.exp(be))
    z = x + bh * h * (x - x0)
    ld = (n - 1) * torch.log(1 + bh * h) + torch.log(1 + bh * h - bh * r / (ea + r) ** 2)
    return z, ld


def maf(layer, x, p, inverse):
    """MAF.forward / inverse (flows_1.py:171-195)."""
    dim = layer.dim
    ip = p["initial_param"]
    cols, ld = [], torch.zeros(x.shape[0], dtype=x.dtype, device=x.device)
    src = x.flip(dims=(1,)) if inverse else x
    for i in range(dim):
        if i == 0:
            mu, alpha = ip[0], ip[1]
        else:
            out = conditioner(layer, p, "layers.%d" % (i - 1),
                              torch.stack(cols, dim=1) if inverse else x[:, :i])
            mu, alpha = out[:, 0], out[:, 1]
        if inverse:
            cols.append(mu + torch.exp(alpha) * src[:, i])
            ld = ld + alpha
        else:
            cols.append((src[:, i] - mu) / torch.exp(alpha))
            ld = ld - alpha
    z = torch.stack(cols, dim=1)
    return (z, ld) if inverse else (z.flip(dims=(1,)), ld)


def actnorm(layer, x, p, inverse):
    """ActNorm.forward / inverse (flows_1.py:207-215); log|det| is a scalar."""
    mu, ls = p["mu"], p["log_sigma"]
    if inverse:
        return (x - mu) / torch.exp(ls), -torch.sum(ls)
    return x * torch.exp(ls) + mu, torch.sum(ls)


def onebyone(layer, x, p, inverse):
    """OneByOneConv.forward / inverse (flows_1.py:235-252)."""
    dim = layer.dim
    L = torch.tril(p["L"], diagonal=-1) + torch.diag(torch.ones(dim, dtype=x.dtype, device=x.device))
    US = torch.triu(p["U"], diagonal=1) + torch.diag(p["S"])
    P = layer.P.to(x.dtype)
    ld = torch.sum(torch.log(torch.abs(p["S"])))
    if inverse:
        return x @ torch.inverse(P @ L @ US), -ld
    return x @ P @ L @ US, ld


def nsf_ar_flows1(layer, x, p, inverse):
    """nf/flows_1.py's NSF_AR (flows_1.py:395-465): net i reads the first i
    coordinates of the INPUT in both directions (a zero column for i = 0),
    through cos/sin(pi v / B) when periodic."""
    dim, K, B = layer.dim, layer.K, layer.B
    cols, ld = [], torch.zeros(x.shape[0], dtype=x.dtype, device=x.device)
    for i in range(dim):
        src = torch.zeros(x.shape[0], 1, dtype=x.dtype, device=x.device) if i == 0 else x[:, :i]
        if layer.periodic:
            src = torch.cat([torch.cos(math.pi * src / B), torch.sin(math.pi * src / B)], dim=-1)
        W, H, D = _nsf_params(conditioner(layer, p, "layers.%d" % i, src), K, B)
        zi, l = unconstrained_rq_spline(x[:, i], W, H, D, inverse, float(B))
        cols.append(zi)
        ld = ld + l
    return torch.stack(cols, dim=1), ld


_BY_CLASS = {"NSF_CL": nsf_cl, "RealNVP": realnvp, "NSF_AR": nsf_ar, "Planar": planar,
             "Radial": radial, "MAF": maf, "ActNorm": actnorm, "OneByOneConv": onebyone}


def layer_forward(layer, x, p, inverse):
    """Dispatch on the layer class (normalizingflow_amd.flows, or a subclass);
    a class naming its restatement in ``_torch_math`` (flows_1.NSF_AR) wins."""
    own = getattr(type(layer), "_torch_math", None)
    if own is not None:
        return globals()[own](layer, x, p, inverse)
    for cls in type(layer).__mro__:
        fn = _BY_CLASS.get(cls.__name__)
        if fn is not None:
            return fn(layer, x, p, inverse)
    raise NotImplementedError("no differentiable restatement for %s" % type(layer).__name__)
