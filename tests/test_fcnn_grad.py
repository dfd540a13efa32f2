"""CPU: the hand-written FCNN recompute-backward (normalizingflow_amd.fcnn_grad,
used by NSF_CL's training backward) against torch autograd through the stock
FCNN (nf/flows.py:20-35), including the split-K weight gradient with a batch
that does not divide into its slices."""
import pytest
import torch

from normalizingflow_amd import fcnn_grad
from normalizingflow_amd.flows import FCNN


@pytest.mark.parametrize("B", [700, 3 * 8192 + 123])
def test_fcnn_vjp_matches_autograd(B):
    torch.manual_seed(0)
    net = FCNN(12, 46, 33).double()
    x = torch.randn(B, 12, dtype=torch.float64, requires_grad=True)
    g = torch.randn(B, 46, dtype=torch.float64)
    out = net(x)
    ref = torch.autograd.grad(out, [x] + list(net.parameters()), g)
    p = {"psi." + n: t.detach() for n, t in net.named_parameters()}
    out2, cache = fcnn_grad.forward_saved(p, "psi.", x.detach())
    torch.testing.assert_close(out2, out.detach())
    gx, grads = fcnn_grad.vjp(p, "psi.", cache, g, True, set(p))
    torch.testing.assert_close(gx, ref[0])
    for (n, _), r in zip(net.named_parameters(), ref[1:]):
        torch.testing.assert_close(grads["psi." + n], r)
    # only some gradients requested
    gx2, grads2 = fcnn_grad.vjp(p, "psi.", cache, g, False, {"psi.network.2.weight"})
    assert gx2 is None and set(grads2) == {"psi.network.2.weight"}


def test_wgrad_split():
    torch.manual_seed(1)
    for B in (100, 8192 * 5, 8192 * 70 + 5):
        g = torch.randn(B, 7, dtype=torch.float64)
        h = torch.randn(B, 3, dtype=torch.float64)
        torch.testing.assert_close(fcnn_grad.wgrad(g, h), g.t() @ h)
