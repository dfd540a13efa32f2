"""GPU: the fused NSF_CL training backward (nfk_fused_nsf_vjp: conditioner
recompute on the matrix cores + the spline VJP in one kernel) against the
unfused backward of the same layer (recompute GEMMs + nfk_rqs_coupling_bwd,
config.USE_FUSED_VJP off) and against the oracle's autograd (nf/flows.py:
227-253, nf/utils.py:58-152 differentiated by torch on the CPU), forward and
inverse, ragged batches, with and without a log|det| gradient.

The two HIP paths differ only in the conditioner logits' last bits (fp16-split
MFMA vs fp32 GEMM recompute), so they agree to fp32 level; the oracle
tolerance is tests/test_gpu_grad.py's (1e-4 of the largest gradient)."""
import pytest
import torch

import nf.flows as nff
from normalizingflow_amd import config
from normalizingflow_amd import kernels as K_
from oracle import nf_oracle as orc

pytestmark = pytest.mark.gpu

# (size, dim, K, hidden, mask): c3 (KBH 3 + tail, K 8), KBH 3 without a tail,
# KBH 2 with K 4, KBH 1 + tail with a ragged last chunk (n_up 12)
SHAPES = [(32, 2, 8, 100, [0]), (32, 2, 8, 96, [1]), (16, 2, 4, 64, [1]), (12, 2, 8, 33, [0])]


def _grads(layer, x, w, v, inverse):
    xd = x.clone().requires_grad_(True)
    z, ld = layer.inverse(xd) if inverse else layer(xd)
    loss = (z * w).sum() + (ld * v).sum()
    params = [p for _, p in layer.named_parameters()]
    return torch.autograd.grad(loss, [xd] + params)


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "s%d_k%d_h%d_m%d" % (s[0], s[2], s[3], s[4][0]))
@pytest.mark.parametrize("inverse", [False, True])
def test_fused_vjp_vs_unfused_and_oracle(shape, inverse, hip_device):
    size, dim, K, hidden, mask = shape
    n_lo, n_up = len(mask) * size, (dim - len(mask)) * size
    assert K_.fused_nsf_vjp_supported(n_lo, n_up, hidden, K)
    torch.manual_seed(11 + size + K + hidden)
    layer = nff.NSF_CL(size=size, dim=dim, K=K, B=3, hidden_dim=hidden, mask=mask)
    sd = {k: v.detach().clone() for k, v in layer.state_dict().items()}
    B = 1000 + 37
    g = torch.Generator().manual_seed(9)
    x = torch.randn(B, size * dim, generator=g) * 1.2
    w = torch.randn(B, size * dim, generator=g)
    v = torch.randn(B, generator=g)
    dev = layer.to(hip_device)
    xd, wd, vd = x.to(hip_device), w.to(hip_device), v.to(hip_device)
    fused = _grads(dev, xd, wd, vd, inverse)
    assert dev.__dict__.get("_vjp_cache") is not None  # the fused backward ran
    prev = config.USE_FUSED_VJP
    config.USE_FUSED_VJP = False
    try:
        plain = _grads(dev, xd, wd, vd, inverse)
    finally:
        config.USE_FUSED_VJP = prev
    names = ["x"] + [n for n, _ in dev.named_parameters()]
    for n, a, b in zip(names, fused, plain):
        scale = float(b.abs().max())
        assert float((a - b).abs().max()) <= 2e-5 * scale + 1e-6, n
    # oracle: autograd through the restatement on the CPU
    xo = x.clone().requires_grad_(True)
    po = {k: t.clone().requires_grad_(True) for k, t in sd.items()}
    zo, ldo = orc.nsf_cl(xo, po, "", size, dim, K, 3, mask, inverse=inverse)
    ref = torch.autograd.grad((zo * w).sum() + (ldo * v).sum(), [xo] + [po[n] for n in names[1:]])
    for n, a, r in zip(names, fused, ref):
        scale = float(r.abs().max())
        assert float((a.cpu() - r).abs().max()) <= 1e-4 * scale, n


def test_fused_vjp_no_logdet_grad(hip_device):
    """gld = None (a loss on z only) and gz = None (a loss on log|det| only)."""
    torch.manual_seed(3)
    layer = nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[1]).to(hip_device)
    x = torch.randn(777, 64, device=hip_device)
    for which in ("z", "ld"):
        xd = x.clone().requires_grad_(True)
        z, ld = layer(xd)
        loss = z.square().sum() if which == "z" else ld.sum()
        got = torch.autograd.grad(loss, [xd] + list(layer.parameters()))
        prev = config.USE_FUSED_VJP
        config.USE_FUSED_VJP = False
        try:
            xd2 = x.clone().requires_grad_(True)
            z2, ld2 = layer(xd2)
            loss2 = z2.square().sum() if which == "z" else ld2.sum()
            ref = torch.autograd.grad(loss2, [xd2] + list(layer.parameters()))
        finally:
            config.USE_FUSED_VJP = prev
        for a, b in zip(got, ref):
            assert float((a - b).abs().max()) <= 2e-5 * float(b.abs().max()) + 1e-6


@pytest.mark.xfail(strict=False, reason="known gap (DESIGN.md section 10.5): at >= 32K rows nfk_fused_nsf_vjp "
                   "gives run-to-run different dL/dparams and dL/dx; cause not found in round 3")
@pytest.mark.parametrize("inverse", [False, True])
def test_fused_vjp_full_occupancy_batch(inverse, hip_device, monkeypatch):
    """Batches large enough that every CU runs the VJP kernel's full complement
    of workgroups at once (2^18 rows; the c3 train step runs 2^20): the fused
    backward should be bitwise reproducible and agree with the unfused path
    (conditioner recompute GEMMs + nfk_rqs_coupling_bwd) at the tolerance of
    the small-batch test.  Round 3 found it is not (tools/dbg_vjp_det.py)."""
    torch.manual_seed(5)
    layer = nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[0]).to(hip_device)
    B = (1 << 18) + 77
    monkeypatch.setattr(config, "FUSED_VJP_MAX_ROWS", B)  # force the fused kernel
    g = torch.Generator(hip_device).manual_seed(4)
    x = torch.randn(B, 64, device=hip_device, generator=g) * 1.2
    w = torch.randn(B, 64, device=hip_device, generator=g)
    v = torch.randn(B, device=hip_device, generator=g)
    a = _grads(layer, x, w, v, inverse)
    b = _grads(layer, x, w, v, inverse)
    for t1, t2 in zip(a, b):
        assert torch.equal(t1, t2)
    prev = config.USE_FUSED_VJP
    config.USE_FUSED_VJP = False
    try:
        plain = _grads(layer, x, w, v, inverse)
    finally:
        config.USE_FUSED_VJP = prev
    names = ["x"] + [n for n, _ in layer.named_parameters()]
    for n, t1, t2 in zip(names, a, plain):
        scale = float(t2.abs().max())
        assert float((t1 - t2).abs().max()) <= 2e-5 * scale + 1e-6, n


def test_large_batch_backward_reproducible(hip_device):
    """The default training backward at 2^18 rows (above
    config.FUSED_VJP_MAX_ROWS: the unfused path) is bitwise reproducible and
    runs without the fused VJP pack."""
    torch.manual_seed(6)
    layer = nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[1]).to(hip_device)
    B = 1 << 18
    assert B > config.FUSED_VJP_MAX_ROWS
    g = torch.Generator(hip_device).manual_seed(8)
    x = torch.randn(B, 64, device=hip_device, generator=g)
    w = torch.randn(B, 64, device=hip_device, generator=g)
    v = torch.randn(B, device=hip_device, generator=g)
    a = _grads(layer, x, w, v, False)
    b = _grads(layer, x, w, v, False)
    assert layer.__dict__.get("_vjp_cache") is None  # the fused kernel did not run
    for t1, t2 in zip(a, b):
        assert torch.equal(t1, t2)
