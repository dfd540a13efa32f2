"""nfk_fcnn_dh (nfk_fcnn_bwd.hip): the FCNN backward's input-gradient GEMMs
with tanh's backward fused, out = (g W) (1 - h^2), on the fp16-split matrix
cores, against fp64 torch.  Error bound per element: 8e-6 of
sum_p |g_bp| * max|W| (the split keeps ~22 bits of each operand relative to its
row / matrix max; fp32 accumulation over P terms adds the rest),
so rows spanning many orders of magnitude, zero rows and ragged batches are
covered; and fcnn_grad.vjp with the kernel equals it with library GEMMs."""
import pytest
import torch

from normalizingflow_amd import config, fcnn_grad
from normalizingflow_amd import kernels as K_

pytestmark = pytest.mark.gpu


def _ref(g, W, h):
    y = g.double() @ W.double()
    if h is not None:
        y = y * (1 - h.double() ** 2)
    # the split's error scale: ~2^-22 of each operand's scale (row max of g,
    # matrix max of W) per product, so sum_p |g_bp| max|W| bounds a row
    bound = g.double().abs().sum(1, keepdim=True) * W.double().abs().max() * torch.ones(1, W.shape[1],
                                                                                       dtype=torch.float64)
    if h is not None:
        bound = bound * (1 - h.double() ** 2).abs()
    return y, bound


@pytest.mark.parametrize("B,P,H,tanh", [(1000, 736, 100, True), (4096, 100, 100, True), (777, 100, 32, False),
                                        (130, 8, 3, True), (64, 36, 128, True), (33, 4, 17, False)])
def test_fcnn_dh_vs_fp64(B, P, H, tanh, hip_device):
    gen = torch.Generator().manual_seed(B + P + H)
    g = torch.randn(B, P, generator=gen)
    # rows over many orders of magnitude, a zero row, a row with one huge entry
    g = g * torch.logspace(-8, 3, B).view(B, 1)[torch.randperm(B, generator=gen)]
    g[B // 3] = 0.0
    g[B // 2, P // 2] = 1e4
    W = torch.randn(P, H, generator=gen) * 0.1
    h = torch.tanh(torch.randn(B, H, generator=gen)) if tanh else None
    ref, bound = _ref(g, W, h)
    gd, Wd = g.to(hip_device), W.to(hip_device)
    hd = None if h is None else h.to(hip_device)
    pack = K_.fcnn_dh_pack(Wd)
    assert pack is not None
    out = torch.empty(B, H, device=hip_device)
    K_.fcnn_dh(gd, pack, (P, H), hd, out)
    err = (out.cpu().double() - ref).abs()
    assert bool((err <= 8e-6 * bound + 1e-30).all()), float((err / (bound + 1e-30)).max())
    assert bool((out[B // 3] == 0).all())


def test_fcnn_dh_strided_h_and_unsupported(hip_device):
    B, P, H = 500, 736, 100
    g = torch.randn(B, P, device=hip_device)
    W = torch.randn(P, H, device=hip_device) * 0.1
    ha = torch.empty(B, 104, device=hip_device)
    ha[:, :H] = torch.tanh(torch.randn(B, H, device=hip_device))
    ha[:, H:] = 1.0
    h = ha[:, :H]
    out = fcnn_grad.dh(g, W, h)
    ref = torch.ops.aten.tanh_backward(g.double() @ W.double(), h.double())
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-5 * float(ref.abs().max()))
    assert K_.fcnn_dh_pack_floats(6, 10) == 0 and K_.fcnn_dh_pack_floats(8, 129) == 0
    # unsupported shapes take the library GEMM
    g2 = torch.randn(10, 6, device=hip_device)
    W2 = torch.randn(6, 5, device=hip_device)
    torch.testing.assert_close(fcnn_grad.dh(g2, W2, None), g2 @ W2)


def test_fcnn_vjp_kernel_vs_library(hip_device):
    torch.manual_seed(3)
    net = torch.nn.Sequential(torch.nn.Linear(32, 100), torch.nn.Tanh(), torch.nn.Linear(100, 100),
                              torch.nn.Tanh(), torch.nn.Linear(100, 736)).to(hip_device)
    p = {"psi.network.%d.%s" % (i, k): getattr(net[i], k).detach() for i in (0, 2, 4) for k in ("weight", "bias")}
    x = torch.randn(3000, 32, device=hip_device)
    _, cache = fcnn_grad.forward_saved(p, "psi.", x)
    g = torch.randn(3000, 736, device=hip_device) * 1e-3
    prev = config.USE_FCNN_DH
    try:
        config.USE_FCNN_DH = True
        gx_k, gr_k = fcnn_grad.vjp(p, "psi.", cache, g, True, set(p))
        config.USE_FCNN_DH = False
        gx_l, gr_l = fcnn_grad.vjp(p, "psi.", cache, g, True, set(p))
    finally:
        config.USE_FCNN_DH = prev
    torch.testing.assert_close(gx_k, gx_l, rtol=1e-4, atol=1e-5 * float(gx_l.abs().max()))
    for k in p:
        torch.testing.assert_close(gr_k[k], gr_l[k], rtol=1e-4, atol=1e-5 * float(gr_l[k].abs().max()))


def test_fcnn_dh_accumulate_into_strided_columns(hip_device):
    """dL/dx of a layer's lower columns added in place into x's gradient
    (columns a, a + st, ...: the single-coordinate NSF_CL masks)."""
    B, P, H = 700, 100, 32
    g = torch.randn(B, P, device=hip_device)
    W = torch.randn(P, H, device=hip_device) * 0.1
    for a, st in ((0, 2), (1, 2), (0, 1)):
        gx = torch.randn(B, 64, device=hip_device)
        ref = gx.clone().double()
        ref[:, a::st][:, :H] += g.double() @ W.double()
        assert fcnn_grad.dh(g, W, None, into=gx[:, a::st][:, :H]) is None
        torch.testing.assert_close(gx.double(), ref, rtol=1e-5, atol=1e-5 * float(ref.abs().max()))


@pytest.mark.parametrize("B,P,H,tanh,strided", [(3000, 32, 100, True, True), (1000, 100, 100, True, False),
                                                (777, 100, 32, False, False), (65, 4, 7, True, False)])
def test_fcnn_linear_vs_fp64(B, P, H, tanh, strided, hip_device):
    """nfk_fcnn_linear, the forward form: act(x W^T + b) against fp64, with the
    split's bound (on the pre-activation; tanh is 1-Lipschitz) plus a few ulps
    of tanhf; x may be a row-strided view (RealNVP's lower half)."""
    gen = torch.Generator().manual_seed(B + P)
    lin = torch.nn.Linear(P, H)
    xs = torch.randn(B, 2 * P if strided else P, generator=gen) * 2
    x = xs[:, :P]
    W, b = lin.weight.detach(), lin.bias.detach()
    pre = x.double() @ W.double().t() + b.double()
    ref = torch.tanh(pre) if tanh else pre
    bound = x.double().abs().sum(1, keepdim=True) * W.double().abs().max()
    xd = xs.to(hip_device)[:, :P]
    Wd, bd = W.to(hip_device), b.to(hip_device)
    out = torch.empty(B, H, device=hip_device)
    K_.fcnn_linear(xd, K_.fcnn_dh_pack(Wd.t()), (P, H), bd, out, tanh=tanh)
    err = (out.cpu().double() - ref).abs()
    assert bool((err <= 8e-6 * bound + 4e-7 * (1 + ref.abs())).all()), float(err.max())


def test_forward_saved_kernel_vs_library(hip_device):
    torch.manual_seed(5)
    net = torch.nn.Sequential(torch.nn.Linear(32, 100), torch.nn.Tanh(), torch.nn.Linear(100, 100),
                              torch.nn.Tanh(), torch.nn.Linear(100, 32)).to(hip_device)
    p = {"s.network.%d.%s" % (i, k): getattr(net[i], k).detach() for i in (0, 2, 4) for k in ("weight", "bias")}
    x = torch.randn(5000, 64, device=hip_device)[:, 32:]
    prev = config.USE_FCNN_FWD
    try:
        config.USE_FCNN_FWD = True
        y_k, c_k = fcnn_grad.forward_saved(p, "s.", x)
        config.USE_FCNN_FWD = False
        y_l, c_l = fcnn_grad.forward_saved(p, "s.", x)
    finally:
        config.USE_FCNN_FWD = prev
    torch.testing.assert_close(y_k, y_l, rtol=1e-5, atol=2e-5 * float(y_l.abs().max()))
    for a, b_ in zip(c_k[1:], c_l[1:]):
        torch.testing.assert_close(a, b_, rtol=1e-5, atol=2e-6)
    with torch.no_grad():
        torch.testing.assert_close(y_l, net(x), rtol=1e-5, atol=1e-5)
