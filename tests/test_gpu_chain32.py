"""GPU parity of the 32x32x16 chain kernel (nfk_fused_chain32.hip, chain form 2
of nfk_fused_nsf_chain): the model's layer loop (nf/models.py:13-29, 37-40)
over c3-class NSF_CL layers (nf/flows.py:227-253: 32 lower inputs, hidden
97-100, K = 8) in one launch, 32 samples per wave.

Its k sums run in another order than the 16x16x32 kernels', so it is checked
against the CPU oracle at the fp32 tolerances of tests/test_gpu_chain.py
(log_prob rtol 1e-5 / atol 1e-4; inverse log|det| atol 3e-4) and against the
16x16 chain (form 1) at the same tolerance, never bitwise; plus ragged batches
(a wave's 32 rows cut anywhere), runs longer than one launch holds, the
accumulated log|det| (mode 2), the reference's no-element-inside error
(nf/utils.py:63) and a forward -> inverse round trip at 2^16 rows.
"""
import pytest
import torch

import nf.flows as nff
import nf.models as nfm
from normalizingflow_amd import _lib, config, flush_status_checks
from normalizingflow_amd import kernels as K_
from oracle import nf_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[2], ids=["f2"])
def form32(request):
    """The 32x32 chain (chain form 2)."""
    lib = _lib.load()
    prev = lib.nfk_debug_chain_form(request.param)
    try:
        lib.form = request.param
        yield lib
    finally:
        lib.nfk_debug_chain_form(prev)


def _model(n_layers, hidden, dev, B=3, scale=1.0, masks=((0,), (1,))):
    torch.manual_seed(1234 + hidden)
    flows = [nff.NSF_CL(size=32, dim=2, K=8, B=B, hidden_dim=hidden, mask=list(masks[i % len(masks)]))
             for i in range(n_layers)]
    if scale != 1.0:
        with torch.no_grad():
            for f in flows:
                for p in f.parameters():
                    p.mul_(scale)
    prior = torch.distributions.MultivariateNormal(torch.zeros(64), torch.eye(64))
    model = nfm.NormalizingFlowModel(prior, flows)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    model = model.to(dev)
    model.prior = torch.distributions.MultivariateNormal(torch.zeros(64, device=dev), torch.eye(64, device=dev))
    return model, sd


def _form(lib, form, fn):
    prev = lib.nfk_debug_chain_form(form)
    try:
        out = fn()
        torch.cuda.synchronize()
        return out, lib.nfk_debug_last_chain_form()
    finally:
        lib.nfk_debug_chain_form(prev)


@pytest.mark.parametrize("n_layers,hidden", [(8, 100), (21, 100), (4, 97), (3, 99)])
@pytest.mark.parametrize("batch", [4096, 1000, 33, 1])
def test_chain32_vs_oracle_and_chain2(n_layers, hidden, batch, form32, hip_device):
    lib = form32
    model, sd = _model(n_layers, hidden, hip_device)
    x = torch.randn(batch, 64, generator=torch.Generator().manual_seed(5 + batch)) * 1.3
    xd = x.to(hip_device)
    with torch.no_grad():
        (lp, f) = _form(lib, lib.form, lambda: model.log_prob(xd))
        assert f == lib.form, "the 32x32 chain did not run"
        (z, pl, ld), _ = _form(lib, lib.form, lambda: model(xd))
        (xi, ldi), _ = _form(lib, lib.form, lambda: model.inverse(xd))
        (lp1, f1) = _form(lib, 1, lambda: model.log_prob(xd))
        assert f1 == 1
        (xi1, ldi1), _ = _form(lib, 1, lambda: model.inverse(xd))
    specs = orc.nsf_cl_specs(n_layers, 32, 2, 8, 3, [[0], [1]])
    ref = orc.model_log_prob(specs, sd, x)
    torch.testing.assert_close(lp.cpu(), ref, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(lp, lp1, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(lp, pl + ld, rtol=2e-7, atol=2e-5)
    xr, ldr = orc.model_inverse(specs, sd, x)
    torch.testing.assert_close(xi.cpu(), xr, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(ldi.cpu(), ldr, rtol=1e-5, atol=3e-4)
    torch.testing.assert_close(xi, xi1, rtol=1e-5, atol=1e-4)
    flush_status_checks()


def test_chain32_one_launch_and_sample(form32, hip_device):
    model, sd = _model(8, 100, hip_device)
    x = torch.randn(512, 64, device=hip_device)
    prev = K_.TIMER
    K_.TIMER = K_.KernelTimer()
    try:
        with torch.no_grad():
            model.log_prob(x)
        torch.cuda.synchronize()
        counts = {k: v[0] for k, v in K_.TIMER.summary().items()}
    finally:
        K_.TIMER = prev
    assert counts == {"nfk_fused_nsf_chain": 1}
    assert form32.nfk_debug_last_chain_form() == form32.form
    torch.manual_seed(7)
    xs, log_px, zs = model.sample(2000)
    specs = orc.nsf_cl_specs(8, 32, 2, 8, 3, [[0], [1]])
    xr, lpr, _ = orc.model_sample_from(specs, sd, zs.cpu())
    torch.testing.assert_close(xs.cpu(), xr, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(log_px.cpu(), lpr, rtol=1e-5, atol=1e-4)


def test_chain32_round_trip(form32, hip_device):
    """inverse(forward(x)) = x and the log|det| cancel, 2^16 rows (a
    size-independent property at a size the oracle would take long on).
    Every layer masks coordinate 0: the reference's NSF_CL writes its output
    as cat([lower, upper]) per particle (nf/flows.py:241, 253), which permutes
    the coordinates for mask [1], so its inverse() undoes forward() only where
    that permutation is the identity."""
    model, _ = _model(8, 100, hip_device, masks=((0,),))
    x = torch.randn(1 << 16, 64, device=hip_device) * 1.2
    with torch.no_grad():
        z, _, ld = model(x)
        xr, ldr = model.inverse(z)
    assert float((xr - x).abs().max()) < 2e-4
    assert float((ld + ldr).abs().max()) < 2e-3
    flush_status_checks()


def test_chain32_large_weights(form32, hip_device):
    """Weights x 8: large logits exercise the power-of-two pre-scaling of the
    pack32 (its own per-layer exponents).  Steep splines make the reference's
    own fp32 log_prob noisy (up to ~1e1 here), so the 32x32 chain is held to
    the 16x16 chain's distance from the oracle rather than a fixed tolerance."""
    model, sd = _model(4, 100, hip_device, scale=8.0)
    x = torch.randn(700, 64, generator=torch.Generator().manual_seed(3)) * 2.0
    with torch.no_grad():
        lp, f = _form(form32, form32.form, lambda: model.log_prob(x.to(hip_device)))
        lp1, f1 = _form(form32, 1, lambda: model.log_prob(x.to(hip_device)))
    assert (f, f1) == (form32.form, 1)
    specs = orc.nsf_cl_specs(4, 32, 2, 8, 3, [[0], [1]])
    ref = orc.model_log_prob(specs, sd, x)
    e2 = (lp.cpu() - ref).abs()
    e1 = (lp1.cpu() - ref).abs()
    assert torch.isfinite(lp).all()
    assert float(e2.max()) <= 2.0 * float(e1.max()) + 1e-3, (float(e2.max()), float(e1.max()))
    assert float(e2.median()) <= 2.0 * float(e1.median()) + 1e-4, (float(e2.median()), float(e1.median()))
    flush_status_checks()


@pytest.mark.parametrize("inverse", [False, True])
def test_chain32_no_element_inside_raises(inverse, form32, hip_device):
    model, _ = _model(4, 100, hip_device)
    x = torch.full((128, 64), 50.0, device=hip_device)
    prev = config.USE_CHAIN
    config.USE_CHAIN = True
    try:
        with pytest.raises(RuntimeError, match="no element inside"):
            with torch.no_grad():
                model.inverse(x) if inverse else model.log_prob(x)
    finally:
        config.USE_CHAIN = prev
    assert form32.nfk_debug_last_chain_form() == form32.form
