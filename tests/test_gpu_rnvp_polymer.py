"""GPU: RealNVP at Polymer_rnvp.yaml's shape -- the configuration the
reference's only Polymer driver loads (applications/examples/polymer.py:29,
applications/input/Polymer_rnvp.yaml:8-9,16-18: 2048 coordinates, hidden 4000,
10 layers, batch 40; the driver's sample(100) and evaluate, polymer.py:37-41).

* forward / both inverses vs the reference's seeded fixture realnvp_d2048_h4000
  (also covered by test_gpu_parity.test_layer_vs_reference_golden);
* a 2-layer model's log_prob vs the oracle at the north star's rtol 1e-5, at
  the config's 40 rows and the driver's 100;
* sample(100): its log_px equals log_prob of the drawn x.
Tolerances as tests/test_gpu_parity.py (z rtol 1e-5 / atol 2e-5, log|det|
rtol 1e-5 / atol 5e-5 with the fp64 fallback of close_or_on_par)."""
import pytest
import torch

import golden_io as gio
import nf.flows as nff
import nf.models as nfm
from normalizingflow_amd import flush_status_checks
from oracle import nf_oracle as orc
from test_gpu_parity import LD_ATOL, LD_RTOL, Z_ATOL, Z_RTOL, close, close_or_on_par

pytestmark = pytest.mark.gpu

VAR = 0.1  # Polymer_rnvp.yaml:24 prior vars


def test_rnvp2048_layer_vs_reference_golden(hip_device):
    meta, d, sd = gio.load("realnvp_d2048_h4000")
    layer = gio.load_into(nff.RealNVP(**meta["kwargs"]), sd).to(hip_device)
    with torch.no_grad():
        z, ld = layer(d["x"].to(hip_device))
        close(z, d["z"], Z_RTOL, Z_ATOL)
        close_or_on_par(ld, d["ld"], d["ld_f64"], LD_RTOL, LD_ATOL)
        xi, ldi = layer.inverse(d["z"].to(hip_device))
        close(xi, d["rt_x"], Z_RTOL, 5e-5)
        close_or_on_par(ldi, d["rt_ld"], d["rt_ld_f64"], LD_RTOL, LD_ATOL)
        xa, lda = layer.inverse(d["x"].to(hip_device))
        close(xa, d["inv_x"], Z_RTOL, 5e-5)
        close_or_on_par(lda, d["inv_ld"], d["inv_ld_f64"], LD_RTOL, LD_ATOL)
    # inverse(forward(x)) = x (RealNVP's inverse is exact, flows.py:65-76)
    assert float((xi - d["x"].to(hip_device)).abs().max()) < 1e-5


@pytest.fixture(scope="module")
def model2(hip_device):
    torch.manual_seed(2048)
    flows = [nff.RealNVP(2048, hidden_dim=4000) for _ in range(2)]
    prior = torch.distributions.MultivariateNormal(torch.zeros(2048), VAR * torch.eye(2048))
    model = nfm.NormalizingFlowModel(prior, flows)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    model = model.to(hip_device)
    model.prior = torch.distributions.MultivariateNormal(torch.zeros(2048, device=hip_device),
                                                        VAR * torch.eye(2048, device=hip_device))
    return model, sd


@pytest.mark.parametrize("rows", [40, 100])
def test_rnvp2048_model_log_prob_vs_oracle(rows, model2, hip_device):
    model, sd = model2
    specs = orc.realnvp_specs(2, 2048)
    x = torch.randn(rows, 2048, generator=torch.Generator().manual_seed(rows)) * VAR ** 0.5
    with torch.no_grad():
        ref = orc.model_log_prob(specs, sd, x, prior_var=VAR)
        lp = model.log_prob(x.to(hip_device))
    close(lp, ref, 1e-5, 1e-5)
    flush_status_checks()


def test_rnvp2048_sample(model2, hip_device):
    model, sd = model2
    xs, lpx, zs = model.sample(100)
    with torch.no_grad():
        lp = model.log_prob(xs)
    close(lpx, lp, 1e-5, 1e-3)
    ref_x, ref_lpx, _ = orc.model_sample_from(orc.realnvp_specs(2, 2048), sd, zs.cpu(), prior_var=VAR)
    close(xs, ref_x, Z_RTOL, 5e-5)
    close(lpx, ref_lpx, 1e-5, 1e-3)
    flush_status_checks()


@pytest.mark.parametrize("rows", [40, 100, 200])
def test_wide_rnvp_chain_bitwise_per_layer(rows, hip_device):
    """Consecutive weight-stream RealNVP layers run as ONE nfk_wide_rnvp_chain
    call (the next layer's input fragments written by the previous layer's
    last coupling, ping-ponged rows): bitwise the per-layer calls, forward
    (log_prob) and inverse (model.inverse), three layers (an odd count: the
    first layer writes z), one launch counted; 200 rows = two row blocks."""
    from normalizingflow_amd import config
    from normalizingflow_amd import kernels as K_
    torch.manual_seed(rows)
    flows = [nff.RealNVP(96, hidden_dim=200) for _ in range(3)]
    prior = torch.distributions.MultivariateNormal(torch.zeros(96), torch.eye(96))
    model = nfm.NormalizingFlowModel(prior, flows).to(hip_device)
    model.prior = torch.distributions.MultivariateNormal(torch.zeros(96, device=hip_device),
                                                        torch.eye(96, device=hip_device))
    x = torch.randn(rows, 96, generator=torch.Generator().manual_seed(7)).to(hip_device)
    with torch.no_grad():
        K_.TIMER = K_.KernelTimer()
        try:
            lp = model.log_prob(x)
            xi, ldi = model.inverse(x)
            torch.cuda.synchronize()
        finally:
            summary, K_.TIMER = K_.TIMER.summary(), None
        assert summary["nfk_wide_rnvp_chain"][0] == 2, summary  # (launches, ...): one per direction
        prev = config.USE_CHAIN
        config.USE_CHAIN = False
        try:
            lp1 = model.log_prob(x)
            xi1, ldi1 = model.inverse(x)
        finally:
            config.USE_CHAIN = prev
    torch.cuda.synchronize()
    assert torch.equal(lp, lp1)
    assert torch.equal(xi, xi1) and torch.equal(ldi, ldi1)
    # a copy after the chained call (its cache holds ctypes pointer arrays)
    import copy
    twin = copy.deepcopy(model)
    with torch.no_grad():
        assert torch.equal(twin.log_prob(x), lp)
    flush_status_checks()


def _lib_path(fn):
    """fn() with the weight-stream path off (library GEMMs + nfk_affine_coupling)."""
    from normalizingflow_amd import config
    prev = config.USE_WIDE_RNVP
    config.USE_WIDE_RNVP = False
    try:
        return fn()
    finally:
        config.USE_WIDE_RNVP = prev


@pytest.mark.parametrize("dim,H,rows", [(2048, 4000, 40), (2048, 4000, 100), (40, 300, 1), (40, 300, 129),
                                        (200, 1000, 256)])
@pytest.mark.parametrize("inverse", [False, True])
def test_wide_rnvp_vs_library_path_and_oracle(dim, H, rows, inverse, hip_device):
    """The weight-stream layer (nfk_wide_rnvp: one call per layer, 128 rows per
    pass) against the library-GEMM path and the oracle, forward and inverse,
    log|det| written (mode 1) and accumulated (mode 2); ragged row counts and
    two-pass batches (129, 256 rows)."""
    from normalizingflow_amd import kernels as K_
    torch.manual_seed(dim + H)
    layer = nff.RealNVP(dim, hidden_dim=H)
    sd = {k: v.detach().clone() for k, v in layer.state_dict().items()}
    layer = layer.to(hip_device)
    x = torch.randn(rows, dim, generator=torch.Generator().manual_seed(rows)) * 0.5
    xd = x.to(hip_device)
    with torch.no_grad():
        assert layer._wide_pack(xd.device, rows) is not None
        K_.TIMER = K_.KernelTimer()
        try:
            z, ld = (layer.inverse if inverse else layer)(xd)
            torch.cuda.synchronize()
            n = {k: v[0] for k, v in K_.TIMER.summary().items()}
        finally:
            K_.TIMER = None
        assert n == {"nfk_wide_rnvp": 1}, n
        zl, ldl = _lib_path(lambda: (layer.inverse if inverse else layer)(xd))
        ref = orc.apply_layer(dict(type="RealNVP", prefix="", dim=dim), x, sd, inverse=inverse)
        # accumulate mode on a preset log|det|
        ld0 = torch.linspace(-2.0, 2.0, rows, device=hip_device)
        z2 = torch.empty_like(xd)
        K_.wide_rnvp(xd, layer._wide_pack(xd.device, rows), z2, logdet=ld0, logdet_mode=2, inverse=inverse)
    close(z, ref[0], Z_RTOL, Z_ATOL)
    close(ld, ref[1], LD_RTOL, LD_ATOL)
    close(zl, ref[0], Z_RTOL, Z_ATOL)
    assert torch.equal(z2, z)
    close(ld0 - torch.linspace(-2.0, 2.0, rows, device=hip_device), ld, 1e-6, 1e-5)


def test_wide_rnvp_reproducible_and_in_place(hip_device):
    """Three runs bitwise equal (split-K partial sums added in a fixed order),
    and z may alias x (each element is read before it is written)."""
    from normalizingflow_amd import kernels as K_
    torch.manual_seed(5)
    layer = nff.RealNVP(2048, hidden_dim=4000).to(hip_device)
    x = torch.randn(100, 2048, device=hip_device) * 0.3
    with torch.no_grad():
        outs = [layer(x) for _ in range(3)]
        for z, ld in outs[1:]:
            assert torch.equal(z, outs[0][0]) and torch.equal(ld, outs[0][1])
        xi = x.clone()
        ld = torch.empty(100, device=hip_device)
        K_.wide_rnvp(xi, layer._wide_pack(x.device, 100), xi, logdet=ld, logdet_mode=1)
    assert torch.equal(xi, outs[0][0]) and torch.equal(ld, outs[0][1])


def test_wide_rnvp_cache_follows_weight_updates(hip_device):
    """An in-place weight update (optimizer step) rebuilds the packs."""
    torch.manual_seed(6)
    layer = nff.RealNVP(64, hidden_dim=512).to(hip_device)
    x = torch.randn(30, 64, device=hip_device)
    with torch.no_grad():
        z0, _ = layer(x)
        layer.t2.network[4].bias.add_(0.25)
        z1, _ = layer(x)
        zl, _ = _lib_path(lambda: layer(x))
    assert not torch.equal(z0, z1)
    close(z1, zl, Z_RTOL, Z_ATOL)
