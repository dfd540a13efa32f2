"""CPU checks of the differentiable restatement used by the recompute-backward
(normalizingflow_amd.torch_math): its values and its gradients (with respect to
the input and every parameter) against the oracle's autograd, for every layer
type, both directions, with inputs reaching into the identity tails; plus an
fp64 finite-difference gradcheck of the spline coupling itself.

The oracle is pinned against the reference's golden vectors
(test_oracle_golden.py), so agreement here ties the training path's
derivatives to the reference's own autograd graph (nf/utils.py:27-152,
nf/flows.py:20-253, nf/flows_1.py:21-97).
"""
import pytest
import torch
import torch.nn.functional as F

from normalizingflow_amd import flows as nff
from normalizingflow_amd import torch_math as tm
from oracle import nf_oracle as orc

GRAD_RTOL, GRAD_ATOL = 1e-4, 1e-5


def _grads(fn, x, params):
    x = x.clone().requires_grad_(True)
    ps = {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}
    z, ld = fn(x, ps)
    torch.manual_seed(1)
    gz = torch.randn_like(z)
    gld = torch.randn_like(ld)
    (z * gz).sum().backward(retain_graph=True)
    (ld * gld).sum().backward()
    return z.detach(), ld.detach(), x.grad, {k: v.grad for k, v in ps.items()}


def _compare(layer, spec_fn, x, inverse, strict_vals=True):
    params = dict(layer.named_parameters())
    z1, l1, gx1, gp1 = _grads(lambda xx, pp: tm.layer_forward(layer, xx, pp, inverse), x, params)
    z2, l2, gx2, gp2 = _grads(lambda xx, pp: spec_fn(xx, {"l." + k: v for k, v in pp.items()},
                                                     inverse), x, params)
    tol = dict(rtol=1e-6, atol=1e-6) if strict_vals else dict(rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(z1, z2, **tol)
    torch.testing.assert_close(l1.expand_as(l2), l2, **tol)
    torch.testing.assert_close(gx1, gx2, rtol=GRAD_RTOL, atol=GRAD_ATOL)
    for k in gp2:
        if gp2[k] is None:
            assert gp1[k] is None or torch.count_nonzero(gp1[k]) == 0, k
            continue
        torch.testing.assert_close(gp1[k], gp2[k], rtol=GRAD_RTOL, atol=GRAD_ATOL, msg=k)


@pytest.mark.parametrize("inverse", [False, True])
@pytest.mark.parametrize("mask", [[0], [1]])
def test_nsf_cl_grads(inverse, mask):
    torch.manual_seed(0)
    L = nff.NSF_CL(size=6, dim=2, K=5, B=3, hidden_dim=24, mask=mask)
    x = torch.randn(40, 12) * 1.8  # ~10% of coordinates in the tails
    spec = lambda xx, sd, inv: orc.nsf_cl(xx, sd, "l.", 6, 2, 5, 3, mask, inverse=inv)
    _compare(L, spec, x, inverse)


def test_nsf_cl_three_coords():
    torch.manual_seed(2)
    L = nff.NSF_CL(size=4, dim=3, K=4, B=2, hidden_dim=16, mask=[1])
    x = torch.randn(30, 12)
    spec = lambda xx, sd, inv: orc.nsf_cl(xx, sd, "l.", 4, 3, 4, 2, [1], inverse=inv)
    _compare(L, spec, x, False)
    _compare(L, spec, x, True)


@pytest.mark.parametrize("inverse", [False, True])
def test_realnvp_grads(inverse):
    torch.manual_seed(3)
    L = nff.RealNVP(dim=8, hidden_dim=20)
    x = torch.randn(32, 8)
    spec = lambda xx, sd, inv: orc.realnvp(xx, sd, "l.", 8, inverse=inv)
    _compare(L, spec, x, inverse)


@pytest.mark.parametrize("inverse", [False, True])
def test_nsf_ar_grads(inverse):
    torch.manual_seed(4)
    L = nff.NSF_AR(dim=4, K=5, B=3, hidden_dim=16)
    x = torch.randn(32, 4) * 1.5
    spec = lambda xx, sd, inv: orc.nsf_ar(xx, sd, "l.", 4, 5, 3, inverse=inv)
    _compare(L, spec, x, inverse)


@pytest.mark.parametrize("nl", ["tanh", "leaky_relu", "elu"])
def test_planar_grads(nl):
    torch.manual_seed(5)
    fn = {"tanh": torch.tanh, "leaky_relu": F.leaky_relu, "elu": F.elu}[nl]
    L = nff.Planar(dim=6, nonlinearity=fn)
    x = torch.randn(32, 6)
    spec = lambda xx, sd, inv: orc.planar(xx, sd, "l.", nl)
    _compare(L, spec, x, False)


def test_radial_grads():
    torch.manual_seed(6)
    L = nff.Radial(dim=6)
    L.reset_parameters(6)
    x = torch.randn(32, 6)
    spec = lambda xx, sd, inv: orc.radial(xx, sd, "l.")
    _compare(L, spec, x, False)


def test_custom_base_network_runs_through_functional_call():
    class Net(torch.nn.Module):
        def __init__(self, i, o, h):
            super().__init__()
            self.a = torch.nn.Linear(i, h)
            self.b = torch.nn.Linear(h, o)

        def forward(self, v):
            return self.b(F.gelu(self.a(v)))

    torch.manual_seed(7)
    L = nff.NSF_CL(size=4, dim=2, K=4, B=3, hidden_dim=12, base_network=Net, mask=[0])
    x = torch.randn(16, 8)
    p = {k: v.detach().clone().requires_grad_(True) for k, v in L.named_parameters()}
    z, ld = tm.layer_forward(L, x, p, False)
    ld.sum().backward()
    # the same layer assembled by hand from the live module
    lower = x.reshape(-1, 4, 2)[:, :, 0]
    raw = L.psi(lower).reshape(-1, 4, 11)
    w, h, d = torch.split(raw, 4, dim=-1)
    up, lad = tm.unconstrained_rq_spline(x.reshape(-1, 4, 2)[:, :, 1], 6 * torch.softmax(w, -1),
                                         6 * torch.softmax(h, -1), F.softplus(d), False, 3.0)
    lad.sum().backward()
    torch.testing.assert_close(ld, lad.sum(1).detach())
    torch.testing.assert_close(z[:, 1::2], up.detach())
    for k, v in L.named_parameters():
        torch.testing.assert_close(p[k].grad, v.grad, msg=k)


def test_spline_gradcheck_fp64():
    torch.manual_seed(8)
    n, K, B = 6, 4, 2.0
    x = (torch.rand(n, 3, dtype=torch.float64) * 5 - 2.5)
    uw = torch.randn(n, 3, K, dtype=torch.float64)
    uh = torch.randn(n, 3, K, dtype=torch.float64)
    ud = torch.randn(n, 3, K - 1, dtype=torch.float64)
    for inverse in (False, True):
        f = lambda a, w, h, d: tm.unconstrained_rq_spline(a, w, h, d, inverse, B)
        assert torch.autograd.gradcheck(f, tuple(t.requires_grad_(True) for t in (x, uw, uh, ud)),
                                        eps=1e-7, atol=1e-6)


def test_layer_fn_plumbing_cpu():
    """flows._LayerFn's gradient bookkeeping (which inputs need grads, the
    [1]-shaped Radial log|det|, parameters without grads) with a CPU stand-in
    for the kernel forward: the node must reproduce plain autograd."""
    class CpuRadial(nff.Radial):
        _vjp = None  # the generic recompute-backward under test (Radial's own VJP is a HIP kernel)

        def _eval(self, x, inverse, status):
            with torch.no_grad():
                return tm.radial(self, x, dict(self.named_parameters()), inverse)

    torch.manual_seed(9)
    L = CpuRadial(5)
    L.reset_parameters(5)
    L.beta.requires_grad_(False)
    x = torch.randn(20, 5)
    named = list(L.named_parameters())
    xa = x.clone().requires_grad_(True)
    z, ld = nff._LayerFn.apply(L, False, None, tuple(n for n, _ in named), xa, *(t for _, t in named))
    (z.sum() + 3 * ld.sum()).backward()
    ga = {k: v.grad.clone() for k, v in L.named_parameters() if v.grad is not None}
    for v in L.parameters():
        v.grad = None
    xb = x.clone().requires_grad_(True)
    z2, ld2 = tm.radial(L, xb, dict(L.named_parameters()), False)
    (z2.sum() + 3 * ld2.sum()).backward()
    torch.testing.assert_close(xa.grad, xb.grad)
    for k, v in L.named_parameters():
        if k == "beta":
            assert v.grad is None and k not in ga
        else:
            torch.testing.assert_close(ga[k], v.grad, msg=k)
    # only the log|det| feeds the loss: gz is None in backward
    xc = x.clone().requires_grad_(True)
    _, ld3 = nff._LayerFn.apply(L, False, None, tuple(n for n, _ in named), xc, *(t for _, t in named))
    ld3.sum().backward()
    assert xc.grad is not None and torch.isfinite(xc.grad).all()


@pytest.mark.parametrize("inverse", [False, True])
def test_maf_actnorm_onebyone_grads(inverse):
    torch.manual_seed(10)
    x = torch.randn(24, 6)
    L = nff.MAF(6, hidden_dim=8)
    _compare(L, lambda xx, sd, inv: orc.maf(xx, sd, "l.", 6, inverse=inv), x, inverse)
    A = nff.ActNorm(6)
    with torch.no_grad():
        A.mu.normal_(0, 0.5)
        A.log_sigma.normal_(0, 0.3)
    _compare(A, lambda xx, sd, inv: orc.actnorm(xx, sd, "l.", inverse=inv), x, inverse)
    np_state = __import__("numpy").random.seed(3)
    C = nff.OneByOneConv(6)
    P = C.P.clone()
    _compare(C, lambda xx, sd, inv: orc.onebyone(xx, dict(sd, **{"l.P": P}), "l.", inverse=inv),
             x, inverse)
    del np_state
