"""CPU oracle for the coupling-layer hot path -- TEST INFRASTRUCTURE ONLY.

This module is the parity checker.  It is imported only by ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py``; the
product path (``normalizingflow_amd`` / ``nf``) never imports it and has no CPU
fallback.

It restates, in plain PyTorch-CPU fp32 (or fp64 when fed fp64 tensors), the
algorithm of the reference ``sherryli59/NormalizingFlow`` for the hot path:

* rational-quadratic spline with linear tails   -> nf/utils.py:20-152
* NSF coupling layer (``NSF_CL``)               -> nf/flows.py:210-253
* affine coupling (``RealNVP``)                  -> nf/flows.py:38-76
* autoregressive spline (``NSF_AR``)             -> nf/flows.py:152-209
* planar / radial flows                          -> nf/flows_1.py:21-97
* MAF / ActNorm / OneByOneConv                    -> nf/flows_1.py:159-252
* MLP conditioner (``FCNN``)                     -> nf/flows.py:20-35
* flow container (``NormalizingFlowModel``)      -> nf/models.py:5-40

The restatement keeps the reference's fp32 operation order (double softmax and
double softplus in NSF_CL, the boundary-derivative constant, the +1e-6 on the
last knot, inclusive tail bounds, the non-prefix-mask output permutation,
Planar's +1e-4, Radial's batch-global norm) but is organised differently: the
boolean compaction of ``unconstrained_RQS`` is replaced by evaluate-everywhere +
select, which is value-identical because every op is per element / per row.

Parity is pinned against golden vectors generated from the reference itself
(``tests/golden/make_golden.py``, fixtures ``tests/golden/*.npz``); see
``tests/test_oracle_golden.py``.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

# nf/utils.py:13-15
MIN_BIN_WIDTH = 1e-3
MIN_BIN_HEIGHT = 1e-3
MIN_DERIVATIVE = 1e-3
KNOT_EPS = 1e-6  # nf/utils.py:20 searchsorted(eps=1e-6)

ERR_NO_INSIDE = "no element inside the spline interval"


# --------------------------------------------------------------------------
# spline pieces (nf/utils.py:58-152)
# --------------------------------------------------------------------------
def _knots(unnorm: torch.Tensor, lo: float, hi: float, min_bin: float):
    """Bin edges and bin sizes from unnormalised logits (utils.py:73-80, 84-91).

    softmax -> floor at ``min_bin`` -> cumulative sum (torch CPU accumulates
    the cumsum in double) -> affine map onto [lo, hi] -> pin both ends -> diff.
    """
    nb = unnorm.shape[-1]
    frac = torch.softmax(unnorm, dim=-1)
    frac = min_bin + (1 - min_bin * nb) * frac
    edges = F.pad(torch.cumsum(frac, dim=-1), pad=(1, 0), mode="constant", value=0.0)
    edges = (hi - lo) * edges + lo
    edges[..., 0] = lo
    edges[..., -1] = hi
    return edges, edges[..., 1:] - edges[..., :-1]


def _bin_of(edges: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """Bin index = #(edges <= v) - 1 with the last edge nudged by +1e-6.

    utils.py:20-25.  The reference nudges the edge tensor in place; the nudged
    edge is never gathered afterwards (index <= K-1), so a copy is equivalent.
    """
    e = edges.clone()
    e[..., -1] += KNOT_EPS
    return (v[..., None] >= e).sum(dim=-1) - 1


def _pick(t: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    return t.gather(-1, idx[..., None])[..., 0]


def rq_spline(inputs, unnormalized_widths, unnormalized_heights, unnormalized_derivatives,
              inverse=False, left=0.0, right=1.0, bottom=0.0, top=1.0,
              min_bin_width=MIN_BIN_WIDTH, min_bin_height=MIN_BIN_HEIGHT,
              min_derivative=MIN_DERIVATIVE):
    """Restatement of ``RQS`` (utils.py:58-152).

    ``unnormalized_derivatives`` carries K+1 entries (already padded).
    Returns ``(outputs, logabsdet, disc_ok)``; ``disc_ok`` is the per-element
    result of the discriminant assertion at utils.py:121 (all True forward).
    """
    nb = unnormalized_widths.shape[-1]
    if min_bin_width * nb > 1.0:
        raise ValueError("Minimal bin width too large for the number of bins")
    if min_bin_height * nb > 1.0:
        raise ValueError("Minimal bin height too large for the number of bins")

    cw, w = _knots(unnormalized_widths, left, right, min_bin_width)
    ch, h = _knots(unnormalized_heights, bottom, top, min_bin_height)
    d = min_derivative + F.softplus(unnormalized_derivatives)

    k = _bin_of(ch if inverse else cw, inputs)
    cw_k, w_k = _pick(cw, k), _pick(w, k)
    ch_k, h_k = _pick(ch, k), _pick(h, k)
    delta_k = _pick(h / w, k)
    d_k = _pick(d, k)
    d_k1 = _pick(d[..., 1:], k)
    slope_gap = d_k + d_k1 - 2 * delta_k

    if inverse:
        y = inputs - ch_k
        qa = y * slope_gap + h_k * (delta_k - d_k)
        qb = h_k * d_k - y * slope_gap
        qc = -delta_k * y
        disc = qb.pow(2) - 4 * qa * qc
        ok = disc >= 0
        root = (2 * qc) / (-qb - torch.sqrt(disc))
        out = root * w_k + cw_k
        th = root
    else:
        th = (inputs - cw_k) / w_k
        ok = torch.ones_like(inputs, dtype=torch.bool)
    t1mt = th * (1 - th)
    denom = delta_k + slope_gap * t1mt
    if not inverse:
        num = h_k * (delta_k * th.pow(2) + d_k * t1mt)
        out = ch_k + num / denom
    dnum = delta_k.pow(2) * (d_k1 * th.pow(2) + 2 * delta_k * t1mt + d_k * (1 - th).pow(2))
    lad = torch.log(dnum) - 2 * torch.log(denom)
    return out, (-lad if inverse else lad), ok


def boundary_derivative_constant(min_derivative=MIN_DERIVATIVE) -> float:
    """utils.py:37-38: log(exp(1 - min_d) - 1), evaluated in float64."""
    return float(np.log(np.exp(1 - min_derivative) - 1))


def unconstrained_rq_spline(inputs, unnormalized_widths, unnormalized_heights,
                            unnormalized_derivatives, inverse=False, tail_bound=1.0,
                            min_bin_width=MIN_BIN_WIDTH, min_bin_height=MIN_BIN_HEIGHT,
                            min_derivative=MIN_DERIVATIVE, strict=True):
    """Restatement of ``unconstrained_RQS`` (utils.py:27-56): identity tails.

    Raises like the reference: RuntimeError when no element is inside
    (torch.min of an empty tensor, utils.py:63) and AssertionError on a negative
    discriminant (utils.py:121), unless ``strict=False``.
    """
    inside = (inputs >= -tail_bound) & (inputs <= tail_bound)
    if strict and not bool(inside.any()):
        raise RuntimeError(ERR_NO_INSIDE)
    c = boundary_derivative_constant(min_derivative)
    dpad = F.pad(unnormalized_derivatives, pad=(1, 1))
    dpad[..., 0] = c
    dpad[..., -1] = c
    # evaluate everywhere on a clamped copy, then select (value-identical to the
    # reference's compaction for the inside elements)
    xin = torch.where(inside, inputs, torch.zeros_like(inputs))
    y, lad, ok = rq_spline(xin, unnormalized_widths, unnormalized_heights, dpad,
                           inverse=inverse, left=-tail_bound, right=tail_bound,
                           bottom=-tail_bound, top=tail_bound,
                           min_bin_width=min_bin_width, min_bin_height=min_bin_height,
                           min_derivative=min_derivative)
    if strict and inverse and not bool(ok[inside].all()):
        raise AssertionError("negative discriminant in RQS inverse")
    out = torch.where(inside, y, inputs)
    lad = torch.where(inside, lad, torch.zeros_like(lad))
    return out, lad


# --------------------------------------------------------------------------
# layers over explicit weights (state-dict tensors)
# --------------------------------------------------------------------------
def fcnn(x, sd, prefix):
    """FCNN (flows.py:20-35): Linear -> tanh -> Linear -> tanh -> Linear."""
    g = lambda n: sd[prefix + n]
    h = torch.tanh(F.linear(x, g("network.0.weight"), g("network.0.bias")))
    h = torch.tanh(F.linear(h, g("network.2.weight"), g("network.2.bias")))
    return F.linear(h, g("network.4.weight"), g("network.4.bias"))


def nsf_cl(x, sd, prefix, size, dim, K, B, mask, inverse=False, strict=True):
    """NSF_CL.forward / inverse (flows.py:227-253).

    lower = masked coordinates of each particle, upper = the rest; the output
    puts the masked coordinates FIRST in every particle group (so a non-prefix
    mask permutes coordinates, and inverse is not forward^-1 then).
    """
    mask = [int(m) for m in mask]
    rest = [c for c in range(dim) if c not in mask]
    g = x.reshape(-1, size, dim)
    lo = g[:, :, mask].flatten(start_dim=1)
    up = g[:, :, rest].flatten(start_dim=1)
    raw = fcnn(lo, sd, prefix + "psi.").reshape(-1, len(rest) * size, 3 * K - 1)
    uw, uh, ud = torch.split(raw, K, dim=2)
    uw = 2 * B * torch.softmax(uw, dim=2)
    uh = 2 * B * torch.softmax(uh, dim=2)
    ud = F.softplus(ud)
    up2, lad = unconstrained_rq_spline(up, uw, uh, ud, inverse=inverse, tail_bound=B,
                                       strict=strict)
    logdet = torch.zeros(x.shape[0], dtype=x.dtype) + lad.sum(dim=1)
    out = torch.cat([lo.reshape(-1, size, len(mask)), up2.reshape(-1, size, len(rest))], dim=2)
    return out.flatten(start_dim=1), logdet


def realnvp(x, sd, prefix, dim, inverse=False):
    """RealNVP.forward / inverse (flows.py:52-76); no clamp on s."""
    half = dim // 2
    a, b = x[:, :half], x[:, half:]
    net = lambda n, v: fcnn(v, sd, prefix + n + ".")
    if not inverse:
        s1 = net("s1", a)
        b = net("t1", a) + b * torch.exp(s1)
        s2 = net("s2", b)
        a = net("t2", b) + a * torch.exp(s2)
        return torch.cat([a, b], dim=1), torch.sum(s1, dim=1) + torch.sum(s2, dim=1)
    s2 = net("s2", b)
    a = (a - net("t2", b)) * torch.exp(-s2)
    s1 = net("s1", a)
    b = (b - net("t1", a)) * torch.exp(-s1)
    return torch.cat([a, b], dim=1), torch.sum(-s1, dim=1) + torch.sum(-s2, dim=1)


def nsf_ar(x, sd, prefix, dim, K, B, inverse=False, strict=True):
    """NSF_AR.forward / inverse (flows.py:175-209): one spline per coordinate,
    conditioned on cos/sin(pi*v[:i]/B) of the preceding coords -- v is the
    input in forward (flows.py:183) but the OUTPUT buffer being filled in
    inverse (flows.py:194,201), i.e. the already-inverted coordinates."""
    n = x.shape[0]
    out = torch.zeros_like(x)
    logdet = torch.zeros(n, dtype=x.dtype)
    pi = torch.tensor(np.pi)
    for i in range(dim):
        if i == 0:
            raw = sd[prefix + "init_param"].expand(n, 3 * K - 1)
        else:
            src = (out if inverse else x)[:, :i]
            feat = torch.cat((torch.cos(pi * src / B), torch.sin(pi * src / B)), axis=-1)
            raw = fcnn(feat, sd, prefix + "layers.%d." % (i - 1))
        uw, uh, ud = torch.split(raw, K, dim=1)
        uw = 2 * B * torch.softmax(uw, dim=1)
        uh = 2 * B * torch.softmax(uh, dim=1)
        ud = F.softplus(ud)
        out[:, i], lad = unconstrained_rq_spline(x[:, i], uw, uh, ud, inverse=inverse,
                                                 tail_bound=B, strict=strict)
        logdet += lad
    return out, logdet


def nsf_ar_flows1(x, sd, prefix, dim, K, B, periodic=True, inverse=False, strict=True):
    """nf/flows_1.py's NSF_AR (its last definition, flows_1.py:395-465): dim
    conditioner nets and no init_param.  Net i reads the INPUT's first i
    coordinates in both directions (x in forward, z in inverse,
    flows_1.py:428-433, 450-455), a zero column for i = 0; periodic=True maps
    them through cos/sin(pi*v/B) first (width 2i, or 2 for i = 0)."""
    n = x.shape[0]
    out = torch.zeros_like(x)
    logdet = torch.zeros(n, dtype=x.dtype)
    pi = torch.tensor(np.pi)
    for i in range(dim):
        src = torch.zeros(n, 1, dtype=x.dtype) if i == 0 else x[:, :i]
        if periodic:
            src = torch.cat((torch.cos(pi * src / B), torch.sin(pi * src / B)), axis=-1)
        raw = fcnn(src, sd, prefix + "layers.%d." % i)
        uw, uh, ud = torch.split(raw, K, dim=1)
        uw = 2 * B * torch.softmax(uw, dim=1)
        uh = 2 * B * torch.softmax(uh, dim=1)
        ud = F.softplus(ud)
        out[:, i], lad = unconstrained_rq_spline(x[:, i], uw, uh, ud, inverse=inverse,
                                                 tail_bound=B, strict=strict)
        logdet += lad
    return out, logdet


_PLANAR_DERIV = {
    # flows_1.py:12-18 (note the reference's -0.01 for leaky_relu's negative side)
    "tanh": lambda v: 1 - torch.pow(torch.tanh(v), 2),
    "leaky_relu": lambda v: (v > 0).type(v.dtype) + (v < 0).type(v.dtype) * -0.01,
    "elu": lambda v: (v > 0).type(v.dtype) + (v < 0).type(v.dtype) * torch.exp(v),
}
_PLANAR_FN = {"tanh": torch.tanh, "leaky_relu": F.leaky_relu, "elu": F.elu}


def planar(x, sd, prefix, nonlinearity="tanh"):
    """Planar.forward (flows_1.py:42-60)."""
    w, u, b = sd[prefix + "w"], sd[prefix + "u"], sd[prefix + "b"]
    if nonlinearity == "tanh":
        wu = w @ u
        uh = u + (torch.log(1 + torch.exp(wu)) - wu - 1) * w / torch.norm(w) ** 2
    else:
        uh = u
    lin = torch.unsqueeze(x @ w, 1) + b
    z = x + uh * _PLANAR_FN[nonlinearity](lin)
    phi = _PLANAR_DERIV[nonlinearity](lin) * w
    return z, torch.log(torch.abs(1 + phi @ uh) + 1e-4)


def radial(x, sd, prefix):
    """Radial.forward (flows_1.py:85-97); r is the Frobenius norm over the
    WHOLE batch, and log_det has shape [1]."""
    x0, la, be = sd[prefix + "x0"], sd[prefix + "log_alpha"], sd[prefix + "beta"]
    n = x.shape[1]
    r = torch.norm(x - x0)
    ea = torch.exp(la)
    h = 1 / (ea + r)
    bh = -ea + torch.log(1 + torch.exp(be))
    z = x + bh * h * (x - x0)
    ld = (n - 1) * torch.log(1 + bh * h) + torch.log(1 + bh * h - bh * r / (ea + r) ** 2)
    return z, ld


def maf(x, sd, prefix, dim, inverse=False):
    """MAF.forward / inverse (flows_1.py:171-195).  Columns are collected and
    stacked instead of written in place (value-identical; keeps autograd valid
    when a conditioner reads the columns already produced)."""
    n = x.shape[0]
    ip = sd[prefix + "initial_param"]
    logdet = torch.zeros(n, dtype=x.dtype)
    src = x.flip(dims=(1,)) if inverse else x
    cols = []
    for i in range(dim):
        if i == 0:
            mu, alpha = ip[0], ip[1]
        else:
            inp = torch.stack(cols, dim=1) if inverse else x[:, :i]
            out = fcnn(inp, sd, prefix + "layers.%d." % (i - 1))
            mu, alpha = out[:, 0], out[:, 1]
        if inverse:
            cols.append(mu + torch.exp(alpha) * src[:, i])
            logdet = logdet + alpha
        else:
            cols.append((src[:, i] - mu) / torch.exp(alpha))
            logdet = logdet - alpha
    z = torch.stack(cols, dim=1)
    return (z, logdet) if inverse else (z.flip(dims=(1,)), logdet)


def actnorm(x, sd, prefix, inverse=False):
    """ActNorm.forward / inverse (flows_1.py:207-215): scalar log|det|."""
    mu, ls = sd[prefix + "mu"], sd[prefix + "log_sigma"]
    if inverse:
        return (x - mu) / torch.exp(ls), -torch.sum(ls)
    return x * torch.exp(ls) + mu, torch.sum(ls)


def onebyone(x, sd, prefix, inverse=False):
    """OneByOneConv.forward / inverse (flows_1.py:235-252).  ``sd[prefix+"P"]``
    must hold the permutation (the reference keeps it outside its state_dict)."""
    Lp, S, Up, P = sd[prefix + "L"], sd[prefix + "S"], sd[prefix + "U"], sd[prefix + "P"]
    dim = S.shape[0]
    L = torch.tril(Lp, diagonal=-1) + torch.diag(torch.ones(dim, dtype=x.dtype))
    U = torch.triu(Up, diagonal=1)
    ld = torch.sum(torch.log(torch.abs(S)))
    if inverse:
        W = P @ L @ (U + torch.diag(S))
        return x @ torch.inverse(W), -ld
    return x @ P @ L @ (U + torch.diag(S)), ld


# --------------------------------------------------------------------------
# model container (nf/models.py:5-40)
# --------------------------------------------------------------------------
def apply_layer(spec, x, sd, inverse=False, strict=True):
    """Dispatch one layer.  ``spec`` = dict(type=..., prefix=..., **ctor args)."""
    t, p = spec["type"], spec["prefix"]
    if t == "NSF_CL":
        return nsf_cl(x, sd, p, spec["size"], spec["dim"], spec["K"], spec["B"], spec["mask"],
                      inverse=inverse, strict=strict)
    if t == "RealNVP":
        return realnvp(x, sd, p, spec["dim"], inverse=inverse)
    if t == "NSF_AR":
        return nsf_ar(x, sd, p, spec["dim"], spec["K"], spec["B"], inverse=inverse, strict=strict)
    if t == "NSF_AR_flows1":
        return nsf_ar_flows1(x, sd, p, spec["dim"], spec["K"], spec["B"],
                             periodic=spec.get("periodic", True), inverse=inverse, strict=strict)
    if t == "Planar":
        if inverse:
            raise NotImplementedError("Planar flow has no algebraic inverse.")
        return planar(x, sd, p, spec.get("nonlinearity", "tanh"))
    if t == "Radial":
        if inverse:
            raise NotImplementedError("Radial flow has no inverse.")
        return radial(x, sd, p)
    if t == "MAF":
        return maf(x, sd, p, spec["dim"], inverse=inverse)
    if t == "ActNorm":
        return actnorm(x, sd, p, inverse=inverse)
    if t == "OneByOneConv":
        return onebyone(x, sd, p, inverse=inverse)
    raise KeyError(t)


def normal_log_prob(z, var=1.0):
    """log N(z; 0, var*I) through torch's MultivariateNormal, exactly as the
    reference's "Normal" prior (applications/src/setup.py:25-30)."""
    d = z.shape[1]
    mvn = torch.distributions.MultivariateNormal(torch.zeros(d, dtype=z.dtype),
                                                 var * torch.eye(d, dtype=z.dtype))
    return mvn.log_prob(z)


def model_forward(specs, sd, x, prior_var=1.0, strict=True):
    """NormalizingFlowModel.forward (models.py:13-20) -> (z, prior_lp, log_det)."""
    logdet = torch.zeros(x.shape[0], dtype=x.dtype)
    for s in specs:
        x, ld = apply_layer(s, x, sd, strict=strict)
        logdet += ld
    return x, normal_log_prob(x, prior_var), logdet


def model_inverse(specs, sd, z, strict=True):
    """NormalizingFlowModel.inverse (models.py:22-29) -> (x, log_det)."""
    logdet = torch.zeros(z.shape[0], dtype=z.dtype)
    for s in specs[::-1]:
        z, ld = apply_layer(s, z, sd, inverse=True, strict=strict)
        logdet += ld
    return z, logdet


def model_log_prob(specs, sd, x, prior_var=1.0, strict=True):
    """NormalizingFlowModel.evaluate (models.py:37-40)."""
    _, plp, ld = model_forward(specs, sd, x, prior_var, strict=strict)
    return plp + ld


def model_sample_from(specs, sd, z, prior_var=1.0, strict=True):
    """NormalizingFlowModel.sample (models.py:31-35) for GIVEN prior draws z."""
    x, ld = model_inverse(specs, sd, z, strict=strict)
    return x, normal_log_prob(z, prior_var) - ld, z


def nsf_cl_specs(n_layers, size, dim, K, B, masks, prefix_fmt="flows.%d."):
    return [dict(type="NSF_CL", prefix=prefix_fmt % i, size=size, dim=dim, K=K, B=B,
                 mask=list(masks[i % len(masks)])) for i in range(n_layers)]


def realnvp_specs(n_layers, dim, prefix_fmt="flows.%d."):
    return [dict(type="RealNVP", prefix=prefix_fmt % i, dim=dim) for i in range(n_layers)]


def log_2pi() -> float:
    return math.log(2 * math.pi)
