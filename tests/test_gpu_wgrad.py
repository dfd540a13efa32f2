"""GPU: nfk_wgrad, the FCNN backward's weight-gradient GEMMs g^T [h | 1] (the
nn.Linear weight and bias gradients of nf/flows.py:20-35 under
applications/src/train.py:26) on bf16 three-way split MFMA.

* against the fp64 product at an fp32-level bound: |err| <= 1e-5 x (|g|^T |h|)
  elementwise, over c3's shapes (736 x 101, 100 x 101, 100 x 32), ragged M,
  N and batch (not a multiple of 32 or of the slice), strided rows, and
  gradients of magnitude 1e-30 (bf16 keeps fp32's exponent: no scaling);
* deterministic: two calls are bitwise equal;
* fcnn_grad.vjp with the kernel (forced on; config.USE_WGRAD_MFMA is off by
  default) vs the split-K library GEMMs at B = 20,000.
"""
import pytest
import torch

from normalizingflow_amd import config, fcnn_grad
from normalizingflow_amd import kernels as K_

pytestmark = pytest.mark.gpu


def _check(g, h, out):
    ref = g.double().t() @ h.double()
    bound = g.double().abs().t() @ h.double().abs()
    err = (out.double() - ref).abs()
    assert bool((err <= 1e-5 * bound + 1e-300).all()), float((err / bound.clamp_min(1e-300)).max())


@pytest.mark.parametrize("B,M,N", [(70000, 736, 101), (40000, 100, 101), (33333, 100, 32),
                                   (1000, 17, 5), (31, 40, 128), (4099, 4096, 1)])
def test_wgrad_vs_fp64(B, M, N, hip_device):
    gen = torch.Generator(device=hip_device).manual_seed(B + M)
    g = torch.randn(B, M, generator=gen, device=hip_device) * torch.rand(B, 1, generator=gen, device=hip_device)
    h = torch.tanh(torch.randn(B, N, generator=gen, device=hip_device))
    out = K_.wgrad(g, h, rows_per_slice=2048)
    assert out.shape == (M, N)
    _check(g, h, out)
    assert torch.equal(out, K_.wgrad(g, h, rows_per_slice=2048))


def test_wgrad_tiny_gradients_and_strided_rows(hip_device):
    gen = torch.Generator(device=hip_device).manual_seed(7)
    wide = torch.randn(9000, 800, generator=gen, device=hip_device) * 1e-30
    g = wide[:, 3:739]  # row stride 800
    hh = torch.tanh(torch.randn(9000, 120, generator=gen, device=hip_device))
    h = hh[:, :101]
    out = K_.wgrad(g, h, rows_per_slice=4096)
    _check(g, h, out)
    assert float(out.abs().max()) > 0


def test_fcnn_vjp_with_and_without_wgrad_kernel(hip_device):
    import nf.flows as nff
    torch.manual_seed(3)
    net = nff.FCNN(32, 736, 100).to(hip_device)
    p = dict(net.named_parameters())
    B = 20000
    x = torch.randn(B, 32, device=hip_device)
    with torch.no_grad():
        h1 = torch.tanh(x @ p["network.0.weight"].t() + p["network.0.bias"])
        h2 = torch.tanh(h1 @ p["network.2.weight"].t() + p["network.2.bias"])
    g = torch.randn(B, 736, device=hip_device) / B
    need = set(p)
    prev = config.USE_WGRAD_MFMA
    try:
        config.USE_WGRAD_MFMA = True
        gx1, gr1 = fcnn_grad.vjp(p, "", (x, h1, h2), g, True, need)
        config.USE_WGRAD_MFMA = False
        gx0, gr0 = fcnn_grad.vjp(p, "", (x, h1, h2), g, True, need)
    finally:
        config.USE_WGRAD_MFMA = prev
    torch.testing.assert_close(gx1, gx0, rtol=0, atol=0)
    for k in need:
        scale = float(gr0[k].abs().max())
        torch.testing.assert_close(gr1[k], gr0[k], rtol=2e-5, atol=2e-6 * scale)
