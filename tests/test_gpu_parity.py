"""GPU parity: the HIP path vs (a) the reference's golden vectors and (b) the
CPU oracle on the same seeded inputs and weights, plus size-independent
properties at the BASELINE sizes.

Tolerances (north star: log_prob within 1e-5 relative, fp32):
  log_prob / prior_lp     rtol 1e-5 (+ atol 1e-5 for values near 0)
  z (elementwise)         rtol 1e-5, atol 2e-5  -- the reference's own fp32 z
                          is off its fp64 value by up to 6.5e-6
  per-layer log|det|      rtol 1e-5, atol 5e-5  (sum of up to 32 terms)
For random / extreme spline parameters (ill-conditioned steep bins) the
criterion is on_par(): >= 99% of elements within the tolerance of the
reference AND our error against the fp64 truth on par with the reference's
own fp32 error (see on_par's docstring).
"""
import pytest
import torch
import torch.nn.functional as F

import golden_io as gio
import nf.flows as nff
import nf.flows_1 as nff1
import nf.models as nfm
import nf.utils as nfu
from normalizingflow_amd import config
from oracle import nf_oracle as orc

pytestmark = pytest.mark.gpu

Z_RTOL, Z_ATOL = 1e-5, 2e-5
LD_RTOL, LD_ATOL = 1e-5, 5e-5
LP_RTOL, LP_ATOL = 1e-5, 1e-5
NL = {"tanh": torch.tanh, "leaky_relu": F.leaky_relu, "elu": F.elu}
DEV = "cuda:0"


def close(a, b, rtol, atol):
    torch.testing.assert_close(a.detach().cpu(), b.detach().cpu(), rtol=rtol, atol=atol)


def on_par(ours, ref, truth, rtol=1e-5, atol=2e-5, within=0.99, factor=4.0):
    """Conditioning-aware parity for random / extreme spline parameters.

    In steep bins a 1-ulp difference of a knot (e.g. device expf vs Sleef's
    exp inside torch's softmax) is amplified by the local slope, for the
    reference as much as for us.  So: (1) >= `within` of the elements agree
    with the reference to rtol/atol, and (2) our error against the fp64
    truth is on par with the reference's own fp32 error (max and p99 within
    `factor`x)."""
    o, r, t = ours.detach().cpu().double(), ref.detach().cpu().double(), truth.double()
    agree = ((o - r).abs() <= atol + rtol * r.abs()).double().mean().item()
    assert agree >= within, "only %.4f of elements within tolerance" % agree
    eo, er = (o - t).abs(), (r - t).abs()
    assert eo.max().item() <= factor * er.max().item() + 1e-6, (eo.max().item(), er.max().item())
    qo, qr = torch.quantile(eo, 0.99).item(), torch.quantile(er, 0.99).item()
    assert qo <= factor * qr + 1e-6, (qo, qr)


def close_or_on_par(ours, ref, truth, rtol, atol, factor=2.0):
    """NSF_AR outputs that sum or chain through hundreds to thousands of
    columns (log|det|: a sum over dim columns; the inverse: conditioned on
    its own outputs): within rtol/atol of the reference, or -- only where the
    fixture holds the fp64 truth -- our max and p99 error against that truth
    within ``factor``x the reference's own fp32 error (the
    reference's fp32 log|det| at Polymer's 2,048 columns is itself 1.4e-4 off
    its fp64 value, a bias that grows with dim)."""
    if truth is not None:
        o, r, t = ours.detach().cpu().double(), ref.detach().cpu().double(), truth.double()
        print("close_or_on_par: max |ours - ref| %.3g; vs fp64 max ours %.3g ref %.3g, p99 ours %.3g ref %.3g"
              % ((o - r).abs().max(), (o - t).abs().max(), (r - t).abs().max(),
                 torch.quantile((o - t).abs().flatten(), 0.99), torch.quantile((r - t).abs().flatten(), 0.99)))
    try:
        close(ours, ref, rtol, atol)
    except AssertionError:
        if truth is None:
            raise
        on_par(ours, ref, truth, rtol, atol, within=0.0, factor=factor)


def build_layer(meta):
    kw = dict(meta["kwargs"])
    if meta["type"] == "Planar":
        kw["nonlinearity"] = NL[meta.get("nonlinearity", "tanh")]
    if meta["type"] == "NSF_AR_flows1":  # nf/flows_1.py:395-465
        return nff1.NSF_AR(**kw)
    return getattr(nff, meta["type"])(**kw)


def spec_of(layer, prefix):
    if isinstance(layer, nff.NSF_CL):
        return dict(type="NSF_CL", prefix=prefix, size=layer.size, dim=layer.dim, K=layer.K,
                    B=layer.B, mask=[int(m) for m in layer.mask])
    if isinstance(layer, nff.RealNVP):
        return dict(type="RealNVP", prefix=prefix, dim=layer.dim)
    if isinstance(layer, nff.NSF_AR):
        return dict(type="NSF_AR", prefix=prefix, dim=layer.dim, K=layer.K, B=layer.B)
    if isinstance(layer, nff.Planar):
        return dict(type="Planar", prefix=prefix, nonlinearity=layer.h.__name__)
    if isinstance(layer, nff.Radial):
        return dict(type="Radial", prefix=prefix)
    if isinstance(layer, nff.MAF):
        return dict(type="MAF", prefix=prefix, dim=layer.dim)
    if isinstance(layer, nff.ActNorm):
        return dict(type="ActNorm", prefix=prefix)
    if isinstance(layer, nff.OneByOneConv):
        return dict(type="OneByOneConv", prefix=prefix)
    raise TypeError(type(layer))


def cpu_sd(module):
    return {k: v.detach().cpu() for k, v in module.state_dict().items()}


# --------------------------------------------------------------------------- golden
LAYERS = [n for n in gio.names() if n.split("_")[0] in ("nsfcl", "realnvp", "planar", "radial", "nsfar",
                                                               "nsfar1", "maf", "actnorm", "onebyone")]


@pytest.mark.parametrize("name", LAYERS)
def test_layer_vs_reference_golden(name, hip_device):
    meta, d, sd = gio.load(name)
    layer = build_layer(meta)
    gio.load_into(layer, sd)
    layer = layer.to(hip_device)
    # the fp64 truth of every output (make_golden.py _f64_run: fp64 log_det
    # accumulator too) in the seeded applications-shape NSF_AR fixtures; the
    # others must agree with the reference outright
    seeded = meta.get("sd_from_seed", False)
    t = {k: d.get(k + "_f64") if seeded else None for k in ("ld", "rt_x", "rt_ld", "inv_x", "inv_ld")}
    with torch.no_grad():
        z, ld = layer(d["x"].to(hip_device))
        close(z, d["z"], Z_RTOL, Z_ATOL)
        close_or_on_par(ld, d["ld"], t["ld"], LD_RTOL, LD_ATOL)
        if "rt_x" in d:
            xi, ldi = layer.inverse(d["z"].to(hip_device))
            close_or_on_par(xi, d["rt_x"], t["rt_x"], Z_RTOL, 5e-5)
            close_or_on_par(ldi, d["rt_ld"], t["rt_ld"], LD_RTOL, LD_ATOL)
            xa, lda = layer.inverse(d["x"].to(hip_device))
            close_or_on_par(xa, d["inv_x"], t["inv_x"], Z_RTOL, 5e-5)
            close_or_on_par(lda, d["inv_ld"], t["inv_ld"], LD_RTOL, LD_ATOL)


def _golden_model(meta, sd, device):
    flows = [build_layer(dict(type=l["type"], kwargs=l["kwargs"])) for l in meta["layers"]]
    d = meta["dim"]
    prior = torch.distributions.MultivariateNormal(torch.zeros(d, device=device),
                                                   meta["var"] * torch.eye(d, device=device))
    model = nfm.NormalizingFlowModel(prior, flows)
    gio.load_into(model, sd, strict=False)
    return model.to(device)


@pytest.mark.parametrize("name", gio.names("model_"))
def test_model_vs_reference_golden(name, hip_device):
    meta, d, sd = gio.load(name)
    model = _golden_model(meta, sd, hip_device)
    x = d["x"].to(hip_device)
    with torch.no_grad():
        z, plp, ld = model(x)
        close(z, d["z"], Z_RTOL, Z_ATOL)
        close(plp, d["prior_lp"], LP_RTOL, LP_ATOL)
        close(ld, d["ld"], LD_RTOL, 1e-4)
        close(model.evaluate(x), d["log_prob"], LP_RTOL, 1e-4)
        close(model.log_prob(x), d["log_prob"], LP_RTOL, 1e-4)
        if "rt_x" in d:
            xi, ldi = model.inverse(d["z"].to(hip_device))
            close(xi, d["rt_x"], Z_RTOL, 5e-5)
            close(ldi, d["rt_ld"], LD_RTOL, 1e-4)
            # sample(): the prior draws differ by device RNG, so feed the
            # reference's draws through our inverse + prior epilogue
            zs = d["sample_z"].to(hip_device)
            xs, lds = model.inverse(zs)
            lp = model._prior_log_prob(zs, logdet=lds, sign=-1)
            close(xs, d["sample_x"], Z_RTOL, 5e-5)
            close(lp, d["sample_log_px"], LP_RTOL, 1e-4)
            xs2, lps2, zs2 = model.sample(64)
            assert xs2.shape == (64, meta["dim"]) and lps2.shape == (64,)
            assert bool(torch.isfinite(lps2).all())


@pytest.mark.parametrize("name", gio.names("rqs_"))
def test_unconstrained_rqs_vs_reference_golden(name, hip_device):
    meta, d, _ = gio.load(name)
    tb = meta["tail_bound"]
    dv = lambda k: d[k].to(hip_device)
    y, lad = nfu.unconstrained_RQS(dv("x"), dv("uw"), dv("uh"), dv("ud"), tail_bound=tb)
    yi, ladi = nfu.unconstrained_RQS(dv("y"), dv("uw"), dv("uh"), dv("ud"), inverse=True,
                                     tail_bound=tb)
    on_par(y, d["y"], d["y_f64"])
    on_par(lad, d["lad"], d["lad_f64"], atol=5e-5)
    y64i, l64i = orc.unconstrained_rq_spline(d["y"].double(), d["uw"].double(), d["uh"].double(),
                                             d["ud"].double(), inverse=True, tail_bound=tb)
    # with scale-3 logits the fp32 quadratic root is catastrophically
    # conditioned: the reference itself is off its fp64 value by up to 0.4
    # there, so only the fp64-error criteria are meaningful (within >= 95%)
    w = 0.95 if meta["scale"] > 2 else 0.99
    on_par(yi, d["inv_y"], y64i, atol=5e-5, within=w)
    on_par(ladi, d["inv_lad"], l64i, atol=5e-5, within=w)


# --------------------------------------------------------------------------- oracle, random
def _c3_model(n_layers=8, size=32, dim=2, K=8, hidden=100, seed=1234):
    torch.manual_seed(seed)
    flows = [nff.NSF_CL(size=size, dim=dim, K=K, B=3, hidden_dim=hidden, mask=[i % 2])
             for i in range(n_layers)]
    D = size * dim
    prior = torch.distributions.MultivariateNormal(torch.zeros(D), torch.eye(D))
    return nfm.NormalizingFlowModel(prior, flows)


def _specs(model):
    return [spec_of(f, "flows.%d." % i) for i, f in enumerate(model.flows)]


def _to_dev(model, device):
    D = model.prior.loc.shape[0]
    var = float(model.prior.covariance_matrix[0, 0])
    model.prior = torch.distributions.MultivariateNormal(torch.zeros(D, device=device),
                                                        var * torch.eye(D, device=device))
    return model.to(device)


@pytest.mark.parametrize("fused", [True, False])
def test_c3_log_prob_vs_oracle(fused, hip_device):
    model = _c3_model()
    sd, specs = cpu_sd(model), _specs(model)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(4096, 64, generator=g)
    ref = orc.model_log_prob(specs, sd, x)
    z_ref, _, ld_ref = orc.model_forward(specs, sd, x)
    model = _to_dev(model, hip_device)
    old = config.USE_FUSED
    config.USE_FUSED = fused
    try:
        with torch.no_grad():
            lp = model.log_prob(x.to(hip_device))
            z, plp, ld = model(x.to(hip_device))
    finally:
        config.USE_FUSED = old
    close(lp, ref, LP_RTOL, LP_ATOL)
    close(z, z_ref, Z_RTOL, 5e-5)
    close(ld, ld_ref, LD_RTOL, 2e-4)


def test_c3_error_vs_fp64(hip_device):
    """the conditioner GEMMs run as the fp16 two-way split
    (22-bit products, fp32 accumulation), not fp32 FMA.  Measured here against
    the fp64 truth (the oracle under default dtype float64) beside the
    reference's own fp32 error (the oracle in fp32) on c3's 8-layer log_prob:
    ours must stay within 2x the reference's max and p99 error, and within
    the bench's 1e-5 relative parity bar."""
    model = _c3_model()
    sd, specs = cpu_sd(model), _specs(model)
    x = torch.randn(4096, 64, generator=torch.Generator().manual_seed(11))
    ref32 = orc.model_log_prob(specs, sd, x)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        ref64 = orc.model_log_prob(specs, {k: v.double() for k, v in sd.items()}, x.double())
    finally:
        torch.set_default_dtype(prev)
    model = _to_dev(model, hip_device)
    with torch.no_grad():
        lp = model.log_prob(x.to(hip_device)).cpu().double()
    e_ours, e_ref = (lp - ref64).abs(), (ref32.double() - ref64).abs()
    print("c3 log_prob vs fp64: max ours %.3g ref %.3g; p99 ours %.3g ref %.3g; max |lp| %.3g"
          % (e_ours.max(), e_ref.max(), torch.quantile(e_ours, 0.99), torch.quantile(e_ref, 0.99),
             ref64.abs().max()))
    assert float(e_ours.max()) <= 2 * float(e_ref.max()) + 1e-6
    assert float(torch.quantile(e_ours, 0.99)) <= 2 * float(torch.quantile(e_ref, 0.99)) + 1e-6
    assert float((e_ours / ref64.abs().clamp_min(1.0)).max()) < 1e-5


@pytest.mark.parametrize("fused", [True, False])
def test_c3_inverse_vs_oracle(fused, hip_device):
    model = _c3_model(n_layers=4)
    sd, specs = cpu_sd(model), _specs(model)
    g = torch.Generator().manual_seed(5)
    z = torch.randn(2048, 64, generator=g)
    x_ref, ld_ref = orc.model_inverse(specs, sd, z)
    model = _to_dev(model, hip_device)
    old = config.USE_FUSED
    config.USE_FUSED = fused
    try:
        x, ld = model.inverse(z.to(hip_device))
    finally:
        config.USE_FUSED = old
    close(x, x_ref, Z_RTOL, 1e-4)
    close(ld, ld_ref, LD_RTOL, 2e-4)


def test_realnvp_c2_vs_oracle(hip_device):
    torch.manual_seed(1234)
    flows = [nff.RealNVP(64, hidden_dim=100) for _ in range(8)]
    prior = torch.distributions.MultivariateNormal(torch.zeros(64), torch.eye(64))
    model = nfm.NormalizingFlowModel(prior, flows)
    sd, specs = cpu_sd(model), _specs(model)
    x = torch.randn(2048, 64, generator=torch.Generator().manual_seed(1))
    ref = orc.model_log_prob(specs, sd, x)
    model = _to_dev(model, hip_device)
    lp = model.log_prob(x.to(hip_device))
    close(lp, ref, LP_RTOL, 1e-4)
    xr, _ = model.inverse(model(x.to(hip_device))[0])
    close(xr, x, 1e-4, 1e-4)


@pytest.mark.parametrize("half,hidden", [(16, 16), (32, 100), (48, 64), (64, 64), (32, 36)])
@pytest.mark.parametrize("inverse", [False, True])
def test_realnvp_fused_layer_vs_oracle(half, hidden, inverse, hip_device):
    """nfk_fused_realnvp (one launch per layer, both half-couplings) against the
    oracle's RealNVP (flows.py:44-76) on one layer, ragged batch, and against
    the unfused HIP path (rocBLAS conditioners + nfk_affine_coupling)."""
    from normalizingflow_amd import config, kernels as K_
    assert K_.fused_realnvp_supported(half, hidden)
    torch.manual_seed(40 + half + hidden)
    layer = nff.RealNVP(2 * half, hidden_dim=hidden)
    x = torch.randn(1000, 2 * half, generator=torch.Generator().manual_seed(3)) * 1.5
    sd = cpu_sd(layer)
    z_ref, ld_ref = orc.realnvp(x, sd, "", 2 * half, inverse=inverse)
    dev = layer.to(hip_device)
    xd = x.to(hip_device)
    with torch.no_grad():
        z, ld = (dev.inverse(xd) if inverse else dev(xd))
        assert dev._pack_cache is not None  # the fused kernel ran
        close(z, z_ref, Z_RTOL, 5e-5)
        close(ld, ld_ref, LD_RTOL, 1e-4)
        config.USE_FUSED = False
        try:
            z2, ld2 = (dev.inverse(xd) if inverse else dev(xd))
        finally:
            config.USE_FUSED = True
        close(z, z2, Z_RTOL, 5e-5)
        close(ld, ld2, LD_RTOL, 1e-4)


@pytest.mark.parametrize("K", [2, 4, 5, 8, 10, 16, 32])
@pytest.mark.parametrize("inverse", [False, True])
def test_unconstrained_rqs_random_vs_oracle(K, inverse, hip_device):
    g = torch.Generator().manual_seed(100 + K)
    n = 3000
    x = torch.randn(n, generator=g) * 2.5
    w, h, d = (torch.randn(n, K, generator=g), torch.randn(n, K, generator=g),
               torch.randn(n, K - 1, generator=g))
    y_ref, l_ref = orc.unconstrained_rq_spline(x, w, h, d, inverse=inverse, tail_bound=3.0)
    y64, l64 = orc.unconstrained_rq_spline(x.double(), w.double(), h.double(), d.double(),
                                           inverse=inverse, tail_bound=3.0)
    y, l = nfu.unconstrained_RQS(*(t.to(hip_device) for t in (x, w, h, d)), inverse=inverse,
                                 tail_bound=3.0)
    on_par(y, y_ref, y64)
    on_par(l, l_ref, l64, atol=5e-5)


def test_rqs_bare_bounds_vs_oracle(hip_device):
    g = torch.Generator().manual_seed(9)
    n, K = 1000, 6
    x = torch.rand(n, generator=g) * 0.98 + 0.01
    w, h, d = (torch.randn(n, K, generator=g), torch.randn(n, K, generator=g),
               torch.randn(n, K + 1, generator=g))
    for inv in (False, True):
        y_ref, l_ref, _ = orc.rq_spline(x, w, h, d, inverse=inv)
        y, l = nfu.RQS(*(t.to(hip_device) for t in (x, w, h, d)), inverse=inv)
        close(y, y_ref, Z_RTOL, 2e-5)
        close(l, l_ref, LD_RTOL, 5e-5)
    with pytest.raises(ValueError, match="outside domain"):
        nfu.RQS((x + 2).to(hip_device), *(t.to(hip_device) for t in (w, h, d)))


def test_searchsorted_side_effect(hip_device):
    loc = torch.tensor([[0.0, 0.5, 1.0], [0.0, 0.25, 1.0]])
    v = torch.tensor([1.0, 0.3])
    ref_loc = loc.clone()
    ref_loc[..., -1] += 1e-6
    ref = (v[..., None] >= ref_loc).sum(-1) - 1
    dl = loc.to(hip_device)
    idx = nfu.searchsorted(dl, v.to(hip_device))
    assert idx.cpu().tolist() == ref.tolist()
    assert torch.equal(dl.cpu(), ref_loc)


@pytest.mark.parametrize("nl", ["tanh", "leaky_relu", "elu"])
def test_planar_random_vs_oracle(nl, hip_device):
    torch.manual_seed(3)
    layer = nff.Planar(37, nonlinearity=NL[nl])
    x = torch.randn(999, 37)
    z_ref, ld_ref = orc.planar(x, cpu_sd(layer), "", nl)
    z, ld = layer.to(hip_device)(x.to(hip_device))
    close(z, z_ref, Z_RTOL, Z_ATOL)
    close(ld, ld_ref, LD_RTOL, LD_ATOL)


def test_radial_random_vs_oracle(hip_device):
    layer = nff.Radial(24)
    torch.manual_seed(4)
    layer.reset_parameters(24)
    x = torch.randn(5000, 24)
    z_ref, ld_ref = orc.radial(x, cpu_sd(layer), "")
    z, ld = layer.to(hip_device)(x.to(hip_device))
    assert ld.shape == (1,)
    close(z, z_ref, Z_RTOL, Z_ATOL)
    close(ld, ld_ref, LD_RTOL, LD_ATOL)


def test_nsf_ar_random_vs_oracle(hip_device):
    torch.manual_seed(8)
    layer = nff.NSF_AR(dim=6, K=8, B=3, hidden_dim=32)
    x = torch.randn(777, 6) * 1.5
    sd = cpu_sd(layer)
    for inv in (False, True):
        z_ref, ld_ref = orc.nsf_ar(x, sd, "", 6, 8, 3, inverse=inv)
        z, ld = (layer.to(hip_device).inverse if inv else layer.to(hip_device))(x.to(hip_device))
        close(z, z_ref, Z_RTOL, 5e-5)
        close(ld, ld_ref, LD_RTOL, LD_ATOL)


# --------------------------------------------------------------------------- edge cases
def test_all_outside_raises_like_reference(hip_device):
    layer = nff.NSF_CL(size=4, dim=2, K=8, B=3, hidden_dim=8, mask=[0]).to(hip_device)
    x = torch.full((16, 8), 10.0, device=hip_device)
    with pytest.raises(RuntimeError):
        layer(x)
    with pytest.raises(RuntimeError):
        layer(torch.zeros(0, 8, device=hip_device))  # empty batch: torch.min of empty
    with pytest.raises(RuntimeError):
        nfu.unconstrained_RQS(torch.full((4,), 9.0, device=hip_device),
                              torch.zeros(4, 8, device=hip_device),
                              torch.zeros(4, 8, device=hip_device),
                              torch.zeros(4, 7, device=hip_device), tail_bound=3.0)


def test_tails_identity_and_boundaries(hip_device):
    n, K = 8, 8
    x = torch.tensor([-3.0, 3.0, -3.0001, 3.0001, 100.0, -100.0, 0.0, 1e-7])
    g = torch.Generator().manual_seed(2)
    w, h, d = torch.randn(n, K, generator=g), torch.randn(n, K, generator=g), torch.randn(n, K - 1, generator=g)
    y, l = nfu.unconstrained_RQS(*(t.to(hip_device) for t in (x, w, h, d)), tail_bound=3.0)
    y_ref, l_ref = orc.unconstrained_rq_spline(x, w, h, d, tail_bound=3.0)
    close(y, y_ref, 0, 2e-6)
    close(l, l_ref, 0, 2e-5)
    assert y.cpu()[2:6].tolist() == x[2:6].tolist() and l.cpu()[2:6].abs().sum() == 0


def test_dim3_masks_and_ragged_batch(hip_device):
    for mask in ([0], [1], [2], [0, 1], [1, 2], [0, 2]):
        torch.manual_seed(11)
        layer = nff.NSF_CL(size=5, dim=3, K=6, B=2.0, hidden_dim=24, mask=mask)
        x = torch.randn(1001, 15)
        z_ref, ld_ref = orc.nsf_cl(x, cpu_sd(layer), "", 5, 3, 6, 2.0, mask)
        z, ld = layer.to(hip_device)(x.to(hip_device))
        close(z, z_ref, Z_RTOL, Z_ATOL)
        close(ld, ld_ref, LD_RTOL, LD_ATOL)


def test_large_n_up_rounds(hip_device):
    # n_up > 256 exercises the multi-round path of the streaming kernel
    torch.manual_seed(12)
    layer = nff.NSF_CL(size=300, dim=2, K=4, B=3, hidden_dim=16, mask=[1])
    x = torch.randn(37, 600)
    z_ref, ld_ref = orc.nsf_cl(x, cpu_sd(layer), "", 300, 2, 4, 3, [1])
    old = config.USE_FUSED
    config.USE_FUSED = False
    try:
        z, ld = layer.to(hip_device)(x.to(hip_device))
    finally:
        config.USE_FUSED = old
    close(z, z_ref, Z_RTOL, Z_ATOL)
    close(ld, ld_ref, LD_RTOL, 2e-4)


# --------------------------------------------------------------------------- full size
def test_c3_full_batch_properties(hip_device):
    """BASELINE c3 at B = 2^20: parity with the oracle on 1,024 random rows and
    the last 65,536 rows (samples are independent), inverse o forward round trip
    for the prefix-mask layers,
    log-det antisymmetry, and run-to-run bitwise determinism."""
    model = _c3_model()
    sd, specs = cpu_sd(model), _specs(model)
    B = 1 << 20
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, 64, generator=g)
    # 1,024 random rows plus a contiguous 64 K slice (the tail-heavy rows of the
    # full batch, 4096 of them beyond |x| = 3 in some coordinate, are covered)
    rows = torch.cat([torch.randperm(B, generator=g)[:1024], torch.arange(B - (1 << 16), B)])
    ref = orc.model_log_prob(specs, sd, x[rows])
    model = _to_dev(model, hip_device)
    xd = x.to(hip_device)
    lp1 = model.log_prob(xd)
    lp2 = model.log_prob(xd)
    assert torch.equal(lp1, lp2)
    close(lp1[rows.to(hip_device)], ref, LP_RTOL, LP_ATOL)
    # a prefix-mask stack is exactly invertible (flows.py:239 keeps the layout)
    torch.manual_seed(7)
    pre = nfm.NormalizingFlowModel(model.prior, [nff.NSF_CL(size=32, dim=2, K=8, B=3,
                                                            hidden_dim=100, mask=[0])
                                                 for _ in range(4)]).to(hip_device)
    with torch.no_grad():
        z, _, ld_f = pre(xd)
        xr, ld_i = pre.inverse(z)
    assert float((xr - xd).abs().max()) < 1e-3
    assert float((ld_f + ld_i).abs().max()) < 1e-3


def test_applications_nsf_cl_branch_vs_oracle(hip_device):
    """The applications' NSF_CL branch (applications/src/setup.py:59-62) at the
    Einstein / LJ / Fe configs' sizes: 32 particles x 3 dims, nsplines 32,
    hidden 354, B = (32 / (8 * 1.28))^(1/3), the six-mask cycle [0], [1], [2],
    [0, 1], [1, 2], [0, 2]: a 6-layer model's log_prob vs the oracle, and
    sample() vs the oracle's inverse of the same prior draws (one k_fused_cl
    launch per layer, tests/test_gpu_cl_wide.py)."""
    torch.manual_seed(21)
    B = (32 / (8 * 1.28)) ** (1.0 / 3.0)
    masks = [[0], [1], [2], [0, 1], [1, 2], [0, 2]]
    flows = [nff.NSF_CL(size=32, dim=3, K=32, B=B, hidden_dim=354, mask=m) for m in masks]
    prior = torch.distributions.MultivariateNormal(torch.zeros(96), torch.eye(96))
    model = nfm.NormalizingFlowModel(prior, flows)
    sd = cpu_sd(model)
    specs = [dict(type="NSF_CL", prefix="flows.%d." % i, size=32, dim=3, K=32, B=B, mask=m)
             for i, m in enumerate(masks)]
    x = torch.randn(300, 96, generator=torch.Generator().manual_seed(4)) * 0.6
    ref = orc.model_log_prob(specs, sd, x)
    model = model.to(hip_device)
    model.prior = torch.distributions.MultivariateNormal(torch.zeros(96, device=hip_device),
                                                        torch.eye(96, device=hip_device))
    lp = model.log_prob(x.to(hip_device))
    close(lp, ref, 1e-5, 2e-4)
    # sample (the inverse chain) vs the oracle's inverse of the same prior draws (the
    # non-prefix masks make inverse and forward not mutually inverse, as in the reference)
    xs, lpx, zs = model.sample(300)
    x_ref, lp_ref, _ = orc.model_sample_from(specs, sd, zs.cpu())
    close(xs, x_ref, 1e-5, 1e-4)
    close(lpx, lp_ref, 1e-5, 2e-4)
