"""GPU parity of the chained RealNVP launch (nfk_fused_realnvp_chain,
k_rnvp_chain in nfk_fused_rnvp.hip): the model's layer loop (nf/models.py:13-29,
37-40) over runs of RealNVP layers (nf/flows.py:44-76) in one launch, x resident
in LDS, the conditioner weights streamed through two LDS slots.

* bitwise equal to one nfk_fused_realnvp launch per layer (config.USE_CHAIN
  off): z, log|det| and the inverse, forward and inverse, ragged batches;
* log_prob as ONE launch with the isotropic-Normal prior as its epilogue;
* against the CPU oracle (restatement of flows.py:44-76, pinned by the
  realnvp_* golden fixtures) at the c2 tolerances of tests/test_gpu_parity.py;
* a NaN input raises the prior's ValueError from the epilogue's status word.
"""
import pytest
import torch

import nf.flows as nff
import nf.models as nfm
from normalizingflow_amd import config
from normalizingflow_amd import kernels as K_
from oracle import nf_oracle as orc

pytestmark = pytest.mark.gpu


def _model(n_layers, dim, hidden, dev, seed=1234):
    torch.manual_seed(seed)
    flows = [nff.RealNVP(dim, hidden_dim=hidden) for _ in range(n_layers)]
    prior = torch.distributions.MultivariateNormal(torch.zeros(dim), torch.eye(dim))
    model = nfm.NormalizingFlowModel(prior, flows)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    model = model.to(dev)
    model.prior = torch.distributions.MultivariateNormal(torch.zeros(dim, device=dev), torch.eye(dim, device=dev))
    return model, sd


def _both(fn):
    prev = config.USE_CHAIN
    try:
        config.USE_CHAIN = True
        a = fn()
        config.USE_CHAIN = False
        b = fn()
    finally:
        config.USE_CHAIN = prev
    return a, b


def _launches(fn):
    prev = K_.TIMER
    K_.TIMER = K_.KernelTimer()
    try:
        fn()
        torch.cuda.synchronize()
        return {k: v[0] for k, v in K_.TIMER.summary().items()}
    finally:
        K_.TIMER = prev


# (layers, dim, hidden): c2 (KBH 3 + tail, two output tiles per half), KBH 2
# without a tail and one output tile, KBH 1 + tail, KBH 3 without a tail
CASES = [(8, 64, 100), (3, 32, 64), (4, 64, 33), (2, 64, 96)]


def test_rnvp_chain_shapes():
    # half_dim <= 32 with hidden <= 128 fits three workgroups per CU; wider
    # layer-1 records (half_dim 48, 64) or KBH 4 run one launch per layer
    assert all(K_.fused_realnvp_chain_max(c[1] // 2, c[2]) > 0 for c in CASES)
    assert K_.fused_realnvp_chain_max(32, 130) == 0 and K_.fused_realnvp_chain_max(64, 100) == 0


@pytest.mark.parametrize("case", CASES, ids=lambda c: "L%d_d%d_h%d" % c)
@pytest.mark.parametrize("batch", [4096, 1000])
def test_rnvp_chain_bitwise_vs_per_layer_and_oracle(case, batch, hip_device):
    n, dim, hidden = case
    assert K_.fused_realnvp_chain_max(dim // 2, hidden) > 0
    model, sd = _model(n, dim, hidden, hip_device)
    x = torch.randn(batch, dim, generator=torch.Generator().manual_seed(5)) * 1.3
    xd = x.to(hip_device)
    with torch.no_grad():
        (zc, plc, ldc), (zs, pls, lds) = _both(lambda: model(xd))
        (lpc,), (lps,) = _both(lambda: (model.log_prob(xd),))
        (xic, ldic), (xis, ldis) = _both(lambda: model.inverse(xd))
    for a, b in ((zc, zs), (plc, pls), (ldc, lds), (xic, xis), (ldic, ldis)):
        assert torch.equal(a, b)
    # log_prob: the prior epilogue sums a row in nfk_normal_logprob's order
    torch.testing.assert_close(lpc, lps, rtol=2e-7, atol=2e-5)
    torch.testing.assert_close(lpc, plc + ldc, rtol=2e-7, atol=2e-5)
    specs = orc.realnvp_specs(n, dim)
    ref = orc.model_log_prob(specs, sd, x)
    torch.testing.assert_close(lpc.cpu(), ref, rtol=1e-5, atol=1e-4)
    xr, ldr = orc.model_inverse(specs, sd, x)
    torch.testing.assert_close(xic.cpu(), xr, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(ldic.cpu(), ldr, rtol=1e-5, atol=3e-4)


def test_c2_log_prob_is_one_launch(hip_device):
    model, _ = _model(8, 64, 100, hip_device)
    x = torch.randn(4096, 64, device=hip_device)
    model.log_prob(x)  # pack
    n = _launches(lambda: model.log_prob(x))
    assert n == {"nfk_fused_realnvp_chain": 1}, n
    with torch.no_grad():  # (under autograd every layer is its own node)
        n = _launches(lambda: model.inverse(x))
    assert n == {"nfk_fused_realnvp_chain": 1}, n


def test_rnvp_chain_roundtrip_and_nan(hip_device):
    model, _ = _model(4, 64, 100, hip_device, seed=7)
    x = torch.randn(3000, 64, device=hip_device)
    with torch.no_grad():
        z, _, ld = model(x)
        xr, ldi = model.inverse(z)
    torch.testing.assert_close(xr, x, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(ldi, -ld, rtol=1e-4, atol=1e-3)
    xn = x.clone()
    xn[17, 3] = float("nan")
    prev = config.STRICT_CHECKS
    config.STRICT_CHECKS = True
    try:
        with pytest.raises(ValueError):
            model.log_prob(xn)
    finally:
        config.STRICT_CHECKS = prev


# half-dimensions the kernels do not take run zero-padded to the next multiple
# of 16 (RealNVP._fused_half): c1's D = 2 (H = 100), D = 6, D = 40 (-> 32)
PAD_CASES = [(4, 2, 100), (3, 6, 64), (2, 40, 100)]


@pytest.mark.parametrize("case", PAD_CASES, ids=lambda c: "L%d_d%d_h%d" % c)
def test_rnvp_padded_halves_vs_oracle(case, hip_device):
    n, dim, hidden = case
    model, sd = _model(n, dim, hidden, hip_device)
    assert model.flows[0]._chain_shape(hip_device)[1] % 16 == 0
    x = torch.randn(3000, dim, generator=torch.Generator().manual_seed(9)) * 1.3
    xd = x.to(hip_device)
    model.log_prob(xd)  # pack
    assert _launches(lambda: model.log_prob(xd)) == {"nfk_fused_realnvp_chain": 1}
    with torch.no_grad():
        (zc, plc, ldc), (zs, pls, lds) = _both(lambda: model(xd))
        (lpc,), (lps,) = _both(lambda: (model.log_prob(xd),))
        (xic, ldic), (xis, ldis) = _both(lambda: model.inverse(xd))
    for a, b in ((zc, zs), (ldc, lds), (xic, xis), (ldic, ldis)):
        assert torch.equal(a, b)
    assert zc.shape == xd.shape and xic.shape == xd.shape
    specs = orc.realnvp_specs(n, dim)
    ref = orc.model_log_prob(specs, sd, x)
    torch.testing.assert_close(lpc.cpu(), ref, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(lps.cpu(), ref, rtol=1e-5, atol=1e-4)
    xr, ldr = orc.model_inverse(specs, sd, x)
    torch.testing.assert_close(xic.cpu(), xr, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(ldic.cpu(), ldr, rtol=1e-5, atol=3e-4)
    # the library-GEMM path (fused kernels off) agrees as well
    prev = config.USE_FUSED
    config.USE_FUSED = False
    try:
        lpu = model.log_prob(xd)
    finally:
        config.USE_FUSED = prev
    torch.testing.assert_close(lpu.cpu(), ref, rtol=1e-5, atol=1e-4)


def test_rnvp_padded_halves_edge_batches(hip_device):
    """Padded halves (D = 2): an empty batch, one row and a column-strided view
    give the oracle's values (the reference accepts all three)."""
    model, sd = _model(4, 2, 100, hip_device)
    specs = orc.realnvp_specs(4, 2)
    assert model.log_prob(torch.empty(0, 2, device=hip_device)).shape == (0,)
    x1 = torch.tensor([[0.3, -1.2]])
    torch.testing.assert_close(model.log_prob(x1.to(hip_device)).cpu(), orc.model_log_prob(specs, sd, x1),
                               rtol=1e-5, atol=1e-5)
    wide = torch.randn(500, 5, generator=torch.Generator().manual_seed(2))
    xv = wide[:, 1:5:2]  # [500, 2] view with row stride 5 and column stride 2
    lp = model.log_prob(wide.to(hip_device)[:, 1:5:2])
    torch.testing.assert_close(lp.cpu(), orc.model_log_prob(specs, sd, xv.contiguous()), rtol=1e-5, atol=1e-5)
    with torch.no_grad():
        z, _, ld = model(wide.to(hip_device)[:, 1:5:2])
    zr, _, ldr = orc.model_forward(specs, sd, xv.contiguous())
    torch.testing.assert_close(z.cpu(), zr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ld.cpu(), ldr, rtol=1e-5, atol=1e-5)
