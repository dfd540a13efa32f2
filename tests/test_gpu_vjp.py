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


def _knot_distance(sd, x, size, dim, K, B, mask, inverse):
    """Per row, the smallest |input - knot| over the row's spline elements, in
    fp64 from the oracle's own pieces (nf/flows.py:231-236, nf/utils.py:73-80)."""
    sd64 = {k: t.double() for k, t in sd.items()}
    rest = [c for c in range(dim) if c not in mask]
    g = x.double().reshape(-1, size, dim)
    lo = g[:, :, mask].flatten(start_dim=1)
    up = g[:, :, rest].flatten(start_dim=1)
    raw = orc.fcnn(lo, sd64, "psi.").reshape(-1, len(rest) * size, 3 * K - 1)
    u = raw[..., K:2 * K] if inverse else raw[..., :K]
    edges, _ = orc._knots(2 * B * torch.softmax(u, dim=2), -B, B, orc.MIN_BIN_WIDTH if not inverse
                          else orc.MIN_BIN_HEIGHT)
    return (up[..., None] - edges).abs().amin(dim=(1, 2))


def _knife_rows(names, got, ref, tol, knife):
    """Rows whose dL/dx differ beyond tol: each must be a knife-edge row, an
    input within 1e-5 (fp64) of a knot, where one path can take the
    neighbouring bin (the two recomputes' logits differ in their last bits) and
    d log f'(x)/dx -- the log|det| part of dL/dx -- jumps (the spline is C1,
    not C2); at most 1 in 10^5 rows may be one.  Returns them (CPU indices)."""
    a, r = got[0].to(ref[0].device), ref[0]
    bad = (a - r).abs() > tol * float(r.abs().max()) + 1e-6
    rows = bad.any(dim=1).nonzero().flatten().cpu()
    if rows.numel():
        assert rows.numel() <= max(1, r.shape[0] // 100000), "%d rows differ" % rows.numel()
        dist = knife(rows)
        assert bool((dist < 1e-5).all()), "differing rows not at a knot: %s" % dist.tolist()
    return rows


def _assert_grads_close(names, got, ref, tol):
    """Every gradient within tol of its largest element."""
    for n, a, r in zip(names, got, ref):
        a = a.to(r.device)
        scale = float(r.abs().max())
        bad = (a - r).abs() > tol * scale + 1e-6
        assert not bool(bad.any()), "%s: %d elements beyond %.1e x max (max diff %.3g, scale %.3g)" % (
            n, int(bad.sum()), tol, float((a - r).abs().max()), scale)


def _compare(names, run_a, run_b, w, v, tol, knife):
    """Gradients of two paths on (w, v)-weighted losses: knife-edge rows
    (_knife_rows) are checked, then zero-weighted (a row with no upstream
    gradient contributes nothing to any gradient, in either path) and every
    gradient is compared on the rest."""
    got, ref = run_a(w, v), run_b(w, v)
    rows = _knife_rows(names, got, ref, tol, knife)
    if rows.numel():
        w, v = w.clone(), v.clone()
        w[rows.to(w.device)] = 0
        v[rows.to(v.device)] = 0
        got, ref = run_a(w, v), run_b(w, v)
    _assert_grads_close(names, got, ref, tol)
    return rows


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


@pytest.mark.parametrize("inverse", [False, True])
def test_fused_vjp_full_occupancy_batch(inverse, hip_device):
    """Batches large enough that every CU runs the VJP kernel's full complement
    of workgroups at once (2^18 rows; the c3 train step runs 2^20): the fused
    backward is bitwise reproducible over three runs and agrees with the
    unfused path (conditioner recompute GEMMs + nfk_rqs_coupling_bwd) at the
    tolerance of the small-batch test.  Round 3 found it was not while the
    kernel was built with packed-FP32 VALU instructions."""
    torch.manual_seed(5)
    layer = nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[0]).to(hip_device)
    B = (1 << 18) + 77
    g = torch.Generator(hip_device).manual_seed(4)
    x = torch.randn(B, 64, device=hip_device, generator=g) * 1.2
    w = torch.randn(B, 64, device=hip_device, generator=g)
    v = torch.randn(B, device=hip_device, generator=g)
    a = _grads(layer, x, w, v, inverse)
    assert layer.__dict__.get("_vjp_cache") is not None  # the fused kernel ran
    for _ in range(2):
        b = _grads(layer, x, w, v, inverse)
        for t1, t2 in zip(a, b):
            assert torch.equal(t1, t2)
    def plain(ww, vv):
        prev = config.USE_FUSED_VJP
        config.USE_FUSED_VJP = False
        try:
            return _grads(layer, x, ww, vv, inverse)
        finally:
            config.USE_FUSED_VJP = prev
    names = ["x"] + [n for n, _ in layer.named_parameters()]
    sd = {k: t.detach().cpu() for k, t in layer.state_dict().items()}
    xc = x.cpu()
    _compare(names, lambda ww, vv: _grads(layer, x, ww, vv, inverse), plain, w, v, 2e-5,
             knife=lambda rows: _knot_distance(sd, xc[rows], 32, 2, 8, 3, [0], inverse))


@pytest.mark.parametrize("inverse", [False, True])
def test_fused_vjp_large_batch_vs_oracle(inverse, hip_device):
    """2^18 rows through the default training backward (the fused kernel at
    full occupancy) against the oracle's autograd (nf/flows.py:227-253,
    nf/utils.py:58-152 differentiated on the CPU, accumulated over 32K-row
    chunks): every gradient within 1e-4 of its largest element."""
    torch.manual_seed(12)
    layer = nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[1])
    sd = {k: t.detach().clone() for k, t in layer.state_dict().items()}
    B = 1 << 18
    g = torch.Generator().manual_seed(13)
    x = torch.randn(B, 64, generator=g) * 1.2
    w = torch.randn(B, 64, generator=g)
    v = torch.randn(B, generator=g)
    dev = layer.to(hip_device)
    names = ["x"] + [n for n, _ in dev.named_parameters()]
    xd = x.to(hip_device)

    def ours(ww, vv):
        g = _grads(dev, xd, ww.to(hip_device), vv.to(hip_device), inverse)
        assert dev.__dict__.get("_vjp_cache") is not None  # the fused kernel ran
        return [t.cpu() for t in g]

    def oracle(ww, vv):
        gx, gp = [], {n: torch.zeros_like(sd[n]) for n in names[1:]}
        for c in range(0, B, 1 << 15):
            xo = x[c:c + (1 << 15)].clone().requires_grad_(True)
            po = {k: t.clone().requires_grad_(True) for k, t in sd.items()}
            zo, ldo = orc.nsf_cl(xo, po, "", 32, 2, 8, 3, [1], inverse=inverse)
            r = torch.autograd.grad((zo * ww[c:c + (1 << 15)]).sum() + (ldo * vv[c:c + (1 << 15)]).sum(),
                                    [xo] + [po[n] for n in names[1:]])
            gx.append(r[0])
            for n, t in zip(names[1:], r[1:]):
                gp[n] += t
        return [torch.cat(gx)] + [gp[n] for n in names[1:]]

    _compare(names, ours, oracle, w, v, 1e-4,
             knife=lambda rows: _knot_distance(sd, x[rows], 32, 2, 8, 3, [1], inverse))


def test_train_batch_backward_reproducible(hip_device):
    """The default training backward at the c3 train batch (2^20 rows, fused
    VJP) is bitwise reproducible over three runs."""
    torch.manual_seed(6)
    layer = nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[1]).to(hip_device)
    B = 1 << 20
    g = torch.Generator(hip_device).manual_seed(8)
    x = torch.randn(B, 64, device=hip_device, generator=g)
    w = torch.randn(B, 64, device=hip_device, generator=g)
    v = torch.randn(B, device=hip_device, generator=g)
    a = _grads(layer, x, w, v, False)
    assert layer.__dict__.get("_vjp_cache") is not None  # the fused kernel ran
    for _ in range(2):
        b = _grads(layer, x, w, v, False)
        for t1, t2 in zip(a, b):
            assert torch.equal(t1, t2)
