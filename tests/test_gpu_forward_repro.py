"""GPU: run-to-run bitwise reproducibility of the FORWARD kernels at full
occupancy (the fused VJP diverged only when waves shared a SIMD, and
the forward kernels ship packed-FP32 code too).  Each kernel runs on at least
2^18 rows -- every wave slot of the chip taken several times over -- three
times on the same inputs; every output must be bitwise the first run's.
Covered: the per-layer fused NSF_CL kernel (k_fused_nsf, c3 shape), the c2
RealNVP per-layer kernel, the fused NSF_AR forward and inverse (Gaussian.yaml's
layer), the wide NSF_CL conditioner (k_fused_cl, the applications' H = 354),
the streaming spline kernel (unfused NSF_CL) and the c5 wide kernel."""
import pytest
import torch

import nf.flows as nff
from normalizingflow_amd import config, flush_status_checks

pytestmark = pytest.mark.gpu

ROWS = (1 << 18) + 77


def _runs(fn, n=3):
    outs = []
    for _ in range(n):
        with torch.no_grad():
            z, ld = fn()
        torch.cuda.synchronize()
        outs.append((z.clone(), ld.clone()))
    return outs


def _assert_same(outs):
    z0, ld0 = outs[0]
    assert torch.isfinite(z0).all() and torch.isfinite(ld0).all()
    for z, ld in outs[1:]:
        assert torch.equal(z, z0), "z differs between runs (max %.3g)" % float((z - z0).abs().max())
        assert torch.equal(ld, ld0), "log|det| differs between runs (max %.3g)" % float((ld - ld0).abs().max())


@pytest.fixture
def no_chain():
    old = config.USE_CHAIN
    config.USE_CHAIN = False
    yield
    config.USE_CHAIN = old


@pytest.mark.parametrize("inverse", [False, True])
def test_fused_nsf_per_layer_reproducible(inverse, hip_device, no_chain):
    torch.manual_seed(1)
    layer = nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[0]).to(hip_device)
    x = torch.randn(ROWS, 64, device=hip_device) * 1.3
    assert layer._fused_pack(x.device) is not None
    _assert_same(_runs(lambda: layer.inverse(x) if inverse else layer(x)))
    flush_status_checks()


@pytest.mark.parametrize("inverse", [False, True])
def test_fused_realnvp_per_layer_reproducible(inverse, hip_device, no_chain):
    torch.manual_seed(2)
    layer = nff.RealNVP(dim=64, hidden_dim=100).to(hip_device)
    x = torch.randn(ROWS, 64, device=hip_device)
    _assert_same(_runs(lambda: layer.inverse(x) if inverse else layer(x)))


@pytest.mark.parametrize("inverse", [False, True])
def test_fused_ar_reproducible(inverse, hip_device):
    torch.manual_seed(3)
    layer = nff.NSF_AR(dim=40, K=10, B=4.0, hidden_dim=80).to(hip_device)
    x = torch.randn(ROWS, 40, device=hip_device) * 1.5
    assert layer._fused_pack(x.device) is not None
    _assert_same(_runs(lambda: layer.inverse(x) if inverse else layer(x)))
    flush_status_checks()


def test_fused_cl_wide_reproducible(hip_device):
    """The applications' NSF_CL conditioner (setup.py:59-62: size 32, dim 3,
    nsplines 32, hidden 354) on 2^16 rows (one 4-wave workgroup per CU)."""
    torch.manual_seed(4)
    layer = nff.NSF_CL(size=32, dim=3, K=32, B=1.5, hidden_dim=354, mask=[0, 1]).to(hip_device)
    x = torch.randn(1 << 16, 96, device=hip_device)
    assert layer._fused_pack(x.device) is not None
    _assert_same(_runs(lambda: layer(x)))
    flush_status_checks()


def test_streaming_spline_reproducible(hip_device):
    """The unfused NSF_CL path: library GEMMs + the streaming spline kernel."""
    old = config.USE_FUSED
    config.USE_FUSED = False
    try:
        torch.manual_seed(5)
        layer = nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[1]).to(hip_device)
        x = torch.randn(ROWS, 64, device=hip_device)
        _assert_same(_runs(lambda: layer(x)))
    finally:
        config.USE_FUSED = old
    flush_status_checks()


def test_wide_nsf_c5_layer_reproducible(hip_device, no_chain):
    torch.manual_seed(6)
    layer = nff.NSF_CL(size=128, dim=2, K=16, B=3, hidden_dim=256, mask=[0]).to(hip_device)
    x = torch.randn(1 << 17, 256, device=hip_device)
    assert layer._fused_pack(x.device) is not None
    _assert_same(_runs(lambda: layer(x)))
    flush_status_checks()


def test_streamed_ar_reproducible(hip_device):
    """The streamed NSF_AR form (k_fused_ar_s, Polymer's kernel; forced on a
    config.py-shaped layer) at 2^16 + 77 rows -- 1,025 row blocks, every CU
    busy several times over -- three runs bitwise equal, the log|det| column
    sum (k_ar_ld_sum) included."""
    from normalizingflow_amd import kernels as K_
    lib = K_._lib.load()
    torch.manual_seed(7)
    layer = nff.NSF_AR(dim=96, K=32, B=1.5, hidden_dim=100).to(hip_device)
    x = torch.randn((1 << 16) + 77, 96, device=hip_device)
    prev = lib.nfk_debug_ar_stream(1)
    try:
        layer.invalidate_caches()
        assert layer._fused_pack(x.device) is not None
        _assert_same(_runs(lambda: layer(x)))
    finally:
        lib.nfk_debug_ar_stream(prev)
        layer.invalidate_caches()
    flush_status_checks()


@pytest.mark.parametrize("dim,B", [(96, (32 / (8 * 1.28)) ** (1.0 / 3.0)), (162, 3 * 2.8841 / 2)])
@pytest.mark.parametrize("inverse", [False, True])
def test_fused_ar_h354_reproducible(dim, B, inverse, hip_device):
    """The one-wave-per-SIMD NSF_AR instances that keep packed FP32 (the
    build rule's exemption, DESIGN.md section 10.5: k_fused_ar<11, ...> at the
    applications' hidden 354 -- Einstein/LJ dim 96, Fe dim 162), forward and
    inverse, at 2^16 + 77 rows: every SIMD of the chip busy several rounds
    over; three runs bitwise equal."""
    torch.manual_seed(8 + dim)
    layer = nff.NSF_AR(dim=dim, K=32, B=B, hidden_dim=354).to(hip_device)
    x = torch.randn((1 << 16) + 77, dim, device=hip_device) * (0.6 * B)
    assert layer._fused_pack(x.device) is not None
    _assert_same(_runs(lambda: layer.inverse(x) if inverse else layer(x)))
    flush_status_checks()
