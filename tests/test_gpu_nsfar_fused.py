"""GPU: the fused NSF_AR layer kernel (nfk_fused_ar.hip, one launch per layer)
against the reference goldens, the CPU oracle and the unfused per-column
path (nf/flows.py:152-209).

Shapes: the reference-generated fixtures nsfar_d4_k4 (H 16),
nsfar_d40_k10_h80 (applications/input/Gaussian.yaml: 20 particles x 2 dims,
nsplines 10, hidden 80, B 4), nsfar_d24_k32_h100 (config.py defaults:
nsplines 32, hidden 100), nsfar_d96_k32_h354 (Einstein / LJ.yaml: 32
particles x 3 dims, nsplines 32, hidden 354) and nsfar_d162_k32_h354
(Fe_*.yaml: 54 particles x 3 dims; both with weights rebuilt from the
fixture's seed), nsfar_d2048_k32_h100 (Polymer.yaml: 2048 x 1, nsplines 32,
hidden 100), plus random ones.  Tolerances: z rtol 1e-5 / atol
2e-5, log|det| rtol 1e-5 / atol 5e-5 (a sum over dim columns), as in
test_gpu_parity.py; the inverse conditions on its own outputs, so it is
compared at 1e-4 absolute where the forward uses 2e-5.  Where a log|det|
(a sum over up to 2,048 columns) misses 5e-5, the fp64 truth decides
(test_gpu_parity.close_or_on_par: our max and p99 error against it within
2x the fp32 reference's own) -- the fixtures' fp64 companions, or the
oracle run in fp64 on the same inputs."""
import pytest
import torch

import golden_io as gio
import nf.flows as nff
import nf.models as nfm
from normalizingflow_amd import config, flush_status_checks
from normalizingflow_amd import kernels as K_
from oracle import nf_oracle as orc
from test_gpu_parity import close_or_on_par

pytestmark = pytest.mark.gpu

Z_RTOL, Z_ATOL = 1e-5, 2e-5
LD_RTOL, LD_ATOL = 1e-5, 5e-5


def close(a, b, rtol, atol):
    torch.testing.assert_close(a.detach().cpu(), b.detach().cpu(), rtol=rtol, atol=atol)


def _sd(layer):
    return {k: v.detach().cpu() for k, v in layer.state_dict().items()}


def _f64(sd):
    return {k: v.double() for k, v in sd.items()}


def _oracle_ar(x, sd, dim, K, B, inverse=False):
    """(out, log|det|) of the oracle in fp32 and its fp64 truth: (o32, l32, o64, l64)."""
    with torch.no_grad():
        o, l = orc.nsf_ar(x, sd, "", dim, K, B, inverse=inverse)
        o64, l64 = orc.nsf_ar(x.double(), _f64(sd), "", dim, K, B, inverse=inverse)
    return o, l, o64, l64


def _launches(fn):
    """(result, {kernel: launches}) of fn() with the per-kernel timer on."""
    K_.TIMER = K_.KernelTimer()
    try:
        out = fn()
        torch.cuda.synchronize()
        summ = K_.TIMER.summary()
    finally:
        K_.TIMER = None
    return out, {k: v[0] for k, v in summ.items()}


@pytest.mark.parametrize("name", ["nsfar_d4_k4", "nsfar_d40_k10_h80", "nsfar_d24_k32_h100", "nsfar_d96_k32_h354",
                                  "nsfar_d162_k32_h354"])
def test_fused_ar_vs_reference_golden(name, hip_device):
    meta, data, sd = gio.load(name)
    kw = meta["kwargs"]
    assert K_.fused_ar_supported(kw["dim"], kw["hidden_dim"], kw["K"])
    layer = gio.load_into(nff.NSF_AR(**kw), sd).to(hip_device)
    x = data["x"].to(hip_device)
    with torch.no_grad():
        (z, ld), n = _launches(lambda: layer(x))
        assert n == {"nfk_fused_ar": 1}, n  # the whole layer is one launch
        close(z, data["z"], Z_RTOL, Z_ATOL)
        close_or_on_par(ld, data["ld"], data.get("ld_f64"), LD_RTOL, LD_ATOL)
        xi, ldi = layer.inverse(z)
        close(xi, data["rt_x"], 1e-5, 1e-4)
        close_or_on_par(ldi, data["rt_ld"], data.get("rt_ld_f64"), LD_RTOL, LD_ATOL)
        xa, lda = layer.inverse(x)
        close(xa, data["inv_x"], 1e-5, 1e-4)
        close_or_on_par(lda, data["inv_ld"], data.get("inv_ld_f64"), LD_RTOL, LD_ATOL)
    flush_status_checks()


@pytest.mark.parametrize("dim,K,H,B,rows", [(40, 10, 80, 4.0, 3000), (17, 8, 100, 3.0, 1000),
                                           (64, 10, 100, 3.0, 2049), (2, 4, 16, 3.0, 77),
                                           (33, 32, 100, 2.5, 640), (96, 32, 354, 1.462, 333),
                                           (96, 32, 100, 1.462, 200)])
def test_fused_ar_vs_oracle_and_unfused(dim, K, H, B, rows, hip_device):
    """Random weights and ragged batches: the fused layer vs the oracle, and
    the unfused per-column path (library GEMMs + nfk_rqs_coupling) vs the
    same oracle."""
    torch.manual_seed(7 + dim)
    layer = nff.NSF_AR(dim=dim, K=K, B=B, hidden_dim=H)
    sd = _sd(layer)
    layer = layer.to(hip_device)
    x = torch.randn(rows, dim, generator=torch.Generator().manual_seed(dim)) * 1.3
    z_ref, ld_ref, _, ld64 = _oracle_ar(x, sd, dim, K, B)
    xi_ref, ldi_ref, _, ldi64 = _oracle_ar(x, sd, dim, K, B, inverse=True)
    xd = x.to(hip_device)
    with torch.no_grad():
        assert layer._fused_pack(xd.device) is not None
        z, ld = layer(xd)
        xi, ldi = layer.inverse(xd)
        prev = config.USE_FUSED
        config.USE_FUSED = False
        try:
            layer.invalidate_caches()
            zu, ldu = layer(xd)
        finally:
            config.USE_FUSED = prev
    close(z, z_ref, Z_RTOL, Z_ATOL)
    close_or_on_par(ld, ld_ref, ld64, LD_RTOL, LD_ATOL)
    close(zu, z_ref, Z_RTOL, Z_ATOL)
    close_or_on_par(ldu, ld_ref, ld64, LD_RTOL, LD_ATOL)
    close(xi, xi_ref, 1e-5, 1e-4)
    close_or_on_par(ldi, ldi_ref, ldi64, LD_RTOL, LD_ATOL)
    flush_status_checks()


def test_fused_ar_round_trip_and_logdet_cancel(hip_device):
    """inverse(forward(x)) = x and the two log|det| cancel, on 2^16 rows of
    the Gaussian.yaml shape (size-independent properties)."""
    torch.manual_seed(3)
    layer = nff.NSF_AR(dim=40, K=10, B=4.0, hidden_dim=80).to(hip_device)
    x = torch.randn(1 << 16, 40, device=hip_device) * 1.5
    with torch.no_grad():
        z, ld = layer(x)
        xr, ldr = layer.inverse(z)
    assert float((xr - x).abs().max()) < 1e-4
    assert float((ld + ldr).abs().max()) < 1e-3
    flush_status_checks()


def test_fused_ar_model_log_prob_and_sample(hip_device):
    """A 3-layer NSF_AR model (config.py's nlayers) through the model API:
    log_prob vs the oracle; sample() draws through the fused inverse and its
    log_px matches log_prob of the drawn x."""
    torch.manual_seed(11)
    flows = [nff.NSF_AR(dim=40, K=10, B=4.0, hidden_dim=80) for _ in range(3)]
    prior = torch.distributions.MultivariateNormal(torch.zeros(40), torch.eye(40))
    model = nfm.NormalizingFlowModel(prior, flows)
    sd = _sd(model)
    specs = [dict(type="NSF_AR", prefix="flows.%d." % i, dim=40, K=10, B=4.0) for i in range(3)]
    x = torch.randn(1024, 40, generator=torch.Generator().manual_seed(2))
    ref = orc.model_log_prob(specs, sd, x)
    model = model.to(hip_device)
    model.prior = torch.distributions.MultivariateNormal(torch.zeros(40, device=hip_device),
                                                        torch.eye(40, device=hip_device))
    (lp, n) = _launches(lambda: model.log_prob(x.to(hip_device)))
    assert n.get("nfk_fused_ar") == 3, n
    close(lp, ref, 1e-5, 1e-4)
    xs, lpx, zs = model.sample(2000)
    lp2 = model.log_prob(xs)
    close(lpx, lp2, 1e-5, 2e-3)
    flush_status_checks()


def test_fused_ar_no_element_inside_raises(hip_device):
    """A column with every element outside [-B, B] raises the reference's
    RuntimeError (torch.min of an empty tensor, utils.py:63)."""
    torch.manual_seed(5)
    layer = nff.NSF_AR(dim=12, K=8, B=3.0, hidden_dim=100).to(hip_device)
    x = torch.randn(500, 12, device=hip_device)
    x[:, 7] = 10.0
    prev = config.STRICT_CHECKS
    config.STRICT_CHECKS = True
    try:
        with torch.no_grad(), pytest.raises(RuntimeError, match="numel"):
            layer(x)
    finally:
        config.STRICT_CHECKS = prev


@pytest.mark.parametrize("dim,K,H,B", [(96, 32, 354, 1.462), (40, 10, 80, 4.0), (24, 32, 100, 3.0),
                                       (96, 32, 100, 1.462)])
@pytest.mark.parametrize("rows", [1, 40, 50, 333, 4096])
def test_fused_ar_column_split_bitwise(dim, K, H, B, rows, hip_device):
    """The forward's column split (small batches: the conditioners spread over
    workgroups, include/nfk.h nfk_fused_ar_ws) gives bitwise the unsplit
    launch's z, log|det| (modes 1 and 2) and status words; the applications'
    batch sizes (40 and 50, applications/input/*.yaml) included."""
    torch.manual_seed(dim + rows)
    layer = nff.NSF_AR(dim=dim, K=K, B=B, hidden_dim=H).to(hip_device)
    x = torch.randn(rows, dim, device=hip_device) * 1.2
    if rows > 1:
        x[0, dim // 2] = 50.0  # one element outside [-B, B]: the identity tail
    pack = layer._fused_pack(x.device)
    assert pack is not None
    if rows <= 333:
        assert K_._lib.load().nfk_fused_ar_workspace(dim, H, K, rows, 0) == dim * rows  # split
    assert K_._lib.load().nfk_fused_ar_workspace(dim, H, K, rows, 1) == 0  # the inverse never splits
    res = {}
    for split in (False, True):
        z = torch.empty_like(x)
        ld1 = torch.full((rows,), 7.0, device=hip_device)
        ld2 = torch.linspace(-3.0, 3.0, rows, device=hip_device)
        st = torch.zeros(dim, dtype=torch.int32, device=hip_device)
        K_.fused_ar(x, pack, dim, H, K, B, z, logdet=ld1, logdet_mode=1, status=st, split=split)
        z2 = torch.empty_like(x)
        K_.fused_ar(x, pack, dim, H, K, B, z2, logdet=ld2, logdet_mode=2, split=split)
        torch.cuda.synchronize()
        assert torch.equal(z, z2)
        res[split] = (z, ld1, ld2, st)
    for a, b in zip(res[False], res[True]):
        assert torch.equal(a, b)
    if rows > 333 or rows < 40:
        return  # (one row: some column has no element inside [-B, B], where the reference raises)
    # and the oracle on the split result
    z_ref, ld_ref, _, ld64 = _oracle_ar(x.cpu(), _sd(layer), dim, K, B)
    close(res[True][0], z_ref, Z_RTOL, Z_ATOL)
    close_or_on_par(res[True][1], ld_ref, ld64, LD_RTOL, LD_ATOL)


@pytest.mark.parametrize("dim,K,H,B,rows", [(96, 32, 354, 1.462, 40), (40, 10, 80, 4.0, 1000), (5, 4, 16, 3.0, 77)])
def test_ar_batched_backward_vs_per_column(dim, K, H, B, rows, hip_device):
    """The forward-direction NSF_AR backward batched over all conditioners
    (NSF_AR._vjp_batched: stacked-weight GEMMs, one spline-VJP launch) against
    the per-column backward (config.AR_BATCHED_VJP_BYTES = 0) and the oracle's
    autograd: dL/dx and every parameter gradient, at the applications' shape
    and batch among others."""
    torch.manual_seed(31 + dim)
    layer = nff.NSF_AR(dim=dim, K=K, B=B, hidden_dim=H)
    sd = _sd(layer)
    layer = layer.to(hip_device)
    x = torch.randn(rows, dim, generator=torch.Generator().manual_seed(dim)) * 0.8
    w = torch.randn(rows, dim, generator=torch.Generator().manual_seed(dim + 1))

    def grads():
        layer.zero_grad(set_to_none=True)
        xd = x.to(hip_device).requires_grad_(True)
        z, ld = layer(xd)
        ((z * w.to(hip_device)).sum() + ld.sum()).backward()
        return [xd.grad.detach().clone()] + [p.grad.detach().clone() for p in layer.parameters()]

    prev = config.AR_BATCHED_VJP_BYTES
    try:
        g_batched = grads()
        config.AR_BATCHED_VJP_BYTES = 0
        g_col = grads()
    finally:
        config.AR_BATCHED_VJP_BYTES = prev
    for a, c in zip(g_batched, g_col):
        scale = float(c.abs().max()) + 1e-12
        torch.testing.assert_close(a.cpu(), c.cpu(), rtol=1e-4, atol=1e-5 * scale)
    # and the oracle's autograd (fp32 restatement) on the same inputs
    xo = x.clone().requires_grad_(True)
    po = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    zo, ldo = orc.nsf_ar(xo, po, "", dim, K, B)
    ((zo * w).sum() + ldo.sum()).backward()
    # (dL/dx sums the chain through up to dim - 1 conditioners: fp32 summation-order
    # differences of a few 1e-4 relative in single elements, for the per-column path too)
    torch.testing.assert_close(g_batched[0].cpu(), xo.grad, rtol=1e-3, atol=5e-5 * float(xo.grad.abs().max()))
    names = [n for n, _ in layer.named_parameters()]
    for n, g in zip(names, g_batched[1:]):
        ref = po[n].grad
        torch.testing.assert_close(g.cpu(), ref, rtol=1e-3, atol=1e-4 * (float(ref.abs().max()) + 1e-12))
    flush_status_checks()


def test_fe162_forward_one_launch_and_speed(hip_device):
    """The Fe configs' layer (Fe_*.yaml: 54 particles x 3 = 162 coordinates,
    nsplines 32, hidden 354, B = 3 * 2.8841 / 2; setup.py:44-58) at their
    50-row batch: ONE fused launch per layer, bitwise the unsplit launch, and
    at least 10x faster than the per-column path (161 conditioners x ~8
    launches)."""
    import time
    B = 3 * 2.8841 / 2
    torch.manual_seed(54)
    layer = nff.NSF_AR(dim=162, K=32, B=B, hidden_dim=354)
    sd = _sd(layer)
    layer = layer.to(hip_device)
    xc = torch.randn(50, 162, generator=torch.Generator().manual_seed(54)) * (0.6 * B)
    x = xc.to(hip_device)
    with torch.no_grad():
        (z, ld), n = _launches(lambda: layer(x))
        assert n == {"nfk_fused_ar": 1}, n

        def timed(fn, reps):
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / reps

        t_fused = timed(lambda: layer(x), 20)
        prev = config.USE_FUSED
        config.USE_FUSED = False
        try:
            layer.invalidate_caches()
            zu, ldu = layer(x)
            t_col = timed(lambda: layer(x), 3)
        finally:
            config.USE_FUSED = prev
            layer.invalidate_caches()
    z_ref, ld_ref, _, ld64 = _oracle_ar(xc, sd, 162, 32, B)
    for zz, ll in ((z, ld), (zu, ldu)):
        close(zz, z_ref, Z_RTOL, Z_ATOL)
        close_or_on_par(ll, ld_ref, ld64, LD_RTOL, LD_ATOL)
    print("fe162 forward at 50 rows: fused %.3f ms, per-column %.3f ms (%.1fx)"
          % (t_fused * 1e3, t_col * 1e3, t_col / t_fused))
    assert t_col >= 10 * t_fused, (t_fused, t_col)
    flush_status_checks()


def test_polymer2048_vs_reference_golden(hip_device):
    """Polymer.yaml's layer (2048 coordinates x 1 dim, nsplines 32, hidden
    config.py:40's 100, B 0.5) at its 40-row batch against the reference's
    fixture: forward, and the inverse of the forward's output and of x."""
    meta, data, sd = gio.load("nsfar_d2048_k32_h100")
    layer = gio.load_into(nff.NSF_AR(**meta["kwargs"]), sd).to(hip_device)
    x = data["x"].to(hip_device)
    with torch.no_grad():
        z, ld = layer(x)
        close(z, data["z"], Z_RTOL, Z_ATOL)
        close_or_on_par(ld, data["ld"], data["ld_f64"], LD_RTOL, LD_ATOL)  # a sum over 2048 columns
        xi, ldi = layer.inverse(z)
        close(xi, data["rt_x"], 1e-5, 1e-4)
        close_or_on_par(ldi, data["rt_ld"], data["rt_ld_f64"], LD_RTOL, LD_ATOL)
        xa, lda = layer.inverse(x)
        close(xa, data["inv_x"], 1e-5, 1e-4)
        close_or_on_par(lda, data["inv_ld"], data["inv_ld_f64"], LD_RTOL, LD_ATOL)
    flush_status_checks()


@pytest.mark.parametrize("dim,rows", [(96, 40), (96, 333), (64, 1000), (23, 64)])
def test_streamed_ar_bitwise_vs_register_form(dim, rows, hip_device):
    """The streamed-layer-1 forward (k_fused_ar_s: the trig operands and the
    layer-1 weights through the LDS slots, k-block-major; the Polymer form)
    forced on shapes the register form also covers (config.py's hidden 100,
    nsplines 32): z, log|det| (modes 1, 2) and the status words bitwise those
    of the register form -- the same products in the same order."""
    lib = K_._lib.load()
    torch.manual_seed(dim + rows)
    layer = nff.NSF_AR(dim=dim, K=32, B=1.5, hidden_dim=100).to(hip_device)
    x = torch.randn(rows, dim, device=hip_device)
    x[0, dim // 3] = 40.0  # one element outside [-B, B]: the identity tail
    res = []
    for force in (0, 1):
        prev = lib.nfk_debug_ar_stream(force)
        try:
            layer.invalidate_caches()
            pack = layer._fused_pack(x.device)
            assert pack is not None
            assert K_.fused_ar_inverse_supported(dim, 100, 32) == (force == 0)
            z = torch.empty_like(x)
            ld1 = torch.full((rows,), 7.0, device=hip_device)
            ld2 = torch.linspace(-3.0, 3.0, rows, device=hip_device)
            st = torch.zeros(dim, dtype=torch.int32, device=hip_device)
            K_.fused_ar(x, pack, dim, 100, 32, 1.5, z, logdet=ld1, logdet_mode=1, status=st)
            z2 = torch.empty_like(x)
            K_.fused_ar(x, pack, dim, 100, 32, 1.5, z2, logdet=ld2, logdet_mode=2)
            torch.cuda.synchronize()
            assert torch.equal(z, z2)
            res.append((z, ld1, ld2, st))
        finally:
            lib.nfk_debug_ar_stream(prev)
            layer.invalidate_caches()
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)


def test_polymer2048_forward_one_launch_and_speed(hip_device):
    """Polymer.yaml's layer at its 40-row batch: the forward is ONE streamed
    launch (plus the trig pre-pass and the column-order log|det| sum), matches
    the oracle, and is far faster than the per-column path (2,047 conditioners
    x ~8 launches)."""
    import time
    torch.manual_seed(2048)
    layer = nff.NSF_AR(dim=2048, K=32, B=0.5, hidden_dim=100)
    sd = _sd(layer)
    layer = layer.to(hip_device)
    x = torch.randn(40, 2048, generator=torch.Generator().manual_seed(5)) * 0.3
    xd = x.to(hip_device)
    assert K_.fused_ar_supported(2048, 100, 32) and not K_.fused_ar_inverse_supported(2048, 100, 32)
    with torch.no_grad():
        (z, ld), n = _launches(lambda: layer(xd))
        assert n == {"nfk_fused_ar": 1}, n
        z_ref, ld_ref, _, ld64 = _oracle_ar(x, sd, 2048, 32, 0.5)
        close(z, z_ref, Z_RTOL, Z_ATOL)
        close_or_on_par(ld, ld_ref, ld64, LD_RTOL, LD_ATOL)

        def timed(fn, reps):
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / reps

        t_fused = timed(lambda: layer(xd), 10)
        prev = config.USE_FUSED
        config.USE_FUSED = False
        try:
            layer.invalidate_caches()
            t_col = timed(lambda: layer(xd), 1)
        finally:
            config.USE_FUSED = prev
            layer.invalidate_caches()
    print("poly2048 forward at 40 rows: fused %.3f ms, per-column %.3f ms (%.1fx)"
          % (t_fused * 1e3, t_col * 1e3, t_col / t_fused))
    assert t_col >= 10 * t_fused, (t_fused, t_col)
    flush_status_checks()


def test_fused_ar_deepcopy_after_forward(hip_device):
    """copy.deepcopy of a layer after a fused forward (its pack cache holds the
    C++ watch): the copy gives bitwise the original's output, and an update to
    the copy's weights changes the copy only."""
    import copy
    torch.manual_seed(9)
    layer = nff.NSF_AR(dim=24, K=8, B=3.0, hidden_dim=64).to(hip_device)
    x = torch.randn(300, 24, device=hip_device)
    with torch.no_grad():
        z, ld = layer(x)
        c = copy.deepcopy(layer)
        zc, ldc = c(x)
        assert torch.equal(z, zc) and torch.equal(ld, ldc)
        c.layers[10].network[4].bias.add_(0.5)
        zc2, _ = c(x)
        z2, ld2 = layer(x)
    assert not torch.equal(zc2, z)
    assert torch.equal(z2, z) and torch.equal(ld2, ld)
    flush_status_checks()


def test_polymer2048_row_blocks_bitwise(hip_device):
    """The streamed form's workspace (~24 KB per row at 2,048 coordinates) is
    capped by config.AR_WORKSPACE_BYTES: a batch over the cap runs as launches
    over row blocks, bitwise the one-launch result; split=False takes the
    workspace too (the streamed shapes have no workspace-free launch)."""
    torch.manual_seed(4)
    layer = nff.NSF_AR(dim=2048, K=32, B=0.5, hidden_dim=100).to(hip_device)
    x = torch.randn(300, 2048, device=hip_device) * 0.3
    pack = layer._fused_pack(x.device)
    per_row = 4 * K_._lib.load().nfk_fused_ar_workspace(2048, 100, 32, 300, 0) / 300
    res = []
    for cap, split, nl in ((1 << 40, True, 1), (int(per_row * 100), True, 5), (1 << 40, False, 1)):
        prev = config.AR_WORKSPACE_BYTES
        config.AR_WORKSPACE_BYTES = cap
        try:
            z = torch.empty_like(x)
            ld = torch.full((300,), 1.5, device=hip_device)
            st = torch.zeros(2048, dtype=torch.int32, device=hip_device)
            (_, n) = _launches(lambda: K_.fused_ar(x, pack, 2048, 100, 32, 0.5, z, logdet=ld, logdet_mode=2,
                                                  status=st, split=split))
        finally:
            config.AR_WORKSPACE_BYTES = prev
        assert n == {"nfk_fused_ar": nl}, (cap, n)
        res.append((z, ld, st))
    for r in res[1:]:
        for a, b in zip(res[0], r):
            assert torch.equal(a, b)


@pytest.mark.parametrize("dim,H,B,rows", [(96, 354, (32 / (8 * 1.28)) ** (1.0 / 3.0), 40),
                                          (162, 354, 3 * 2.8841 / 2, 50), (2048, 100, 0.5, 40)])
def test_fused_ar_app_model_log_prob(dim, H, B, rows, hip_device):
    """A 2-layer NSF_AR model at the applications' shapes (Einstein/LJ dim 96,
    Fe dim 162, Polymer dim 2048) and their training batches: log_prob
    (models.py:37-40) against the oracle at the north star's rtol 1e-5, and
    our error against the oracle's fp64 run within 2x the oracle's own fp32
    error where the 1e-5 agreement is not bitwise."""
    torch.manual_seed(dim + 1)
    flows = [nff.NSF_AR(dim=dim, K=32, B=B, hidden_dim=H) for _ in range(2)]
    model = nfm.NormalizingFlowModel(torch.distributions.MultivariateNormal(torch.zeros(dim), torch.eye(dim)),
                                     flows)
    sd = _sd(model)
    specs = [dict(type="NSF_AR", prefix="flows.%d." % i, dim=dim, K=32, B=B) for i in range(2)]
    x = torch.randn(rows, dim, generator=torch.Generator().manual_seed(dim)) * (0.6 * B)
    with torch.no_grad():
        ref = orc.model_log_prob(specs, sd, x)
        ref64 = orc.model_log_prob(specs, _f64(sd), x.double())
    model = model.to(hip_device)
    model.prior = torch.distributions.MultivariateNormal(torch.zeros(dim, device=hip_device),
                                                        torch.eye(dim, device=hip_device))
    (lp, n) = _launches(lambda: model.log_prob(x.to(hip_device)))
    assert n.get("nfk_fused_ar") == 2, n
    close(lp, ref, 1e-5, 1e-5)
    e_ours = float((lp.cpu().double() - ref64).abs().max())
    e_ref = float((ref.double() - ref64).abs().max())
    print("dim %d log_prob: max |ours - fp64| %.3g, max |oracle fp32 - fp64| %.3g" % (dim, e_ours, e_ref))
    assert e_ours <= 2 * e_ref + 1e-5 * float(ref64.abs().max()), (e_ours, e_ref)
    flush_status_checks()


@pytest.mark.parametrize("dim,K,rows", [(96, 32, 77), (40, 32, 40), (130, 32, 5)])
def test_ar_seqinv_vs_oracle(dim, K, rows, hip_device):
    """The library-driven column-by-column inverse (nfk_ar_seqinv: the layers
    whose inverse the fused register form does not take; forced here with the
    streamed form on config.py-shaped layers) against the oracle's inverse,
    ragged batches over two 64-row passes, log|det| modes 1 and 2, an element
    outside [-B, B] (the identity tail), run-to-run bitwise."""
    lib = K_._lib.load()
    torch.manual_seed(dim + K)
    layer = nff.NSF_AR(dim=dim, K=K, B=1.5, hidden_dim=100)
    sd = _sd(layer)
    layer = layer.to(hip_device)
    z = torch.randn(rows, dim, generator=torch.Generator().manual_seed(rows)) * 0.7
    z[0, dim // 3] = 9.0
    xi_ref, ldi_ref, _, ldi64 = _oracle_ar(z, sd, dim, K, 1.5, inverse=True)
    zd = z.to(hip_device)
    prev = lib.nfk_debug_ar_stream(1)
    try:
        layer.invalidate_caches()
        assert not K_.fused_ar_inverse_supported(dim, 100, K)
        with torch.no_grad():
            (res, n) = _launches(lambda: layer.inverse(zd))
            assert n == {"nfk_ar_seqinv": 1}, n
            xi, ldi = res
            xi2, ldi2 = layer.inverse(zd)
            ld0 = torch.linspace(-1.0, 1.0, rows, device=hip_device)
            out = torch.empty_like(zd)
            st = torch.zeros(dim, dtype=torch.int32, device=hip_device)
            keep = layer._pack_cache[3]
            K_.ar_seqinv(zd, keep[3], keep[1], dim, 100, K, 1.5, out, logdet=ld0, logdet_mode=2, status=st)
    finally:
        lib.nfk_debug_ar_stream(prev)
        layer.invalidate_caches()
    assert torch.equal(xi, xi2) and torch.equal(ldi, ldi2)
    close(xi, xi_ref, 1e-5, 1e-4)
    close_or_on_par(ldi, ldi_ref, ldi64, LD_RTOL, LD_ATOL)
    assert torch.equal(out, xi)
    close(ld0 - torch.linspace(-1.0, 1.0, rows, device=hip_device), ldi, 1e-6, 1e-5)
    assert int(st[dim // 3]) & 1 and all(int(v) & 1 for v in st.cpu())  # NFK_ST_INSIDE_SEEN in every column


@pytest.mark.parametrize("dim,K,H,rows", [(20, 8, 16, 33), (37, 10, 37, 70), (70, 4, 128, 64), (12, 16, 64, 5)])
def test_ar_seqinv_shapes_vs_oracle(dim, K, H, rows, hip_device):
    """nfk_ar_seqinv over its supported range, called directly with the
    layer's own Linear pointers: hidden widths 16 / 37 (not a multiple of 4:
    the element-wise weight loads) / 64 / 128 (the maximum), K 4 / 8 / 10 / 16,
    against the oracle's inverse; one and two 64-row passes."""
    import ctypes
    assert K_.ar_seqinv_supported(dim, H, K)
    torch.manual_seed(1000 + dim + H)
    layer = nff.NSF_AR(dim=dim, K=K, B=1.5, hidden_dim=H)
    sd = _sd(layer)
    layer = layer.to(hip_device)
    z = torch.randn(rows, dim, generator=torch.Generator().manual_seed(rows + H)) * 0.7
    xi_ref, ldi_ref, _, ldi64 = _oracle_ar(z, sd, dim, K, 1.5, inverse=True)
    flat = [t.detach().contiguous() for m in layer._stock_linears() for t in (m.weight, m.bias)]
    assert len(flat) == 6 * (dim - 1)
    ptrs = (ctypes.c_void_p * len(flat))(*[t.data_ptr() for t in flat])
    zd = z.to(hip_device)
    out = torch.empty_like(zd)
    ld = torch.zeros(rows, device=hip_device)
    st = torch.zeros(dim, dtype=torch.int32, device=hip_device)
    with torch.no_grad():
        K_.ar_seqinv(zd, ptrs, layer.init_param.detach().contiguous(), dim, H, K, 1.5, out, logdet=ld,
                     logdet_mode=1, status=st)
        out2 = torch.empty_like(zd)
        K_.ar_seqinv(zd, ptrs, layer.init_param.detach().contiguous(), dim, H, K, 1.5, out2, logdet=None,
                     logdet_mode=0)
    torch.cuda.synchronize()
    close(out, xi_ref, 1e-5, 1e-4)
    close_or_on_par(ld, ldi_ref, ldi64, LD_RTOL, LD_ATOL)
    assert torch.equal(out, out2)
    assert all(int(v) & 1 for v in st.cpu())


def test_polymer2048_inverse_speed(hip_device):
    """Polymer.yaml's layer inverted at the 40-row batch: the library-driven
    column loop (nfk_ar_seqinv) bitwise-run-to-run, close to the per-column host
    path, and timed against it."""
    import time
    from normalizingflow_amd import config as cfg
    torch.manual_seed(2049)
    layer = nff.NSF_AR(dim=2048, K=32, B=0.5, hidden_dim=100).to(hip_device)
    z = torch.randn(40, 2048, device=hip_device) * 0.2

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    with torch.no_grad():
        xs, lds = layer.inverse(z)
        t_seq = timed(lambda: layer.inverse(z), 3)
        prev = cfg.USE_AR_SEQINV
        cfg.USE_AR_SEQINV = False
        try:
            xc, ldc = layer.inverse(z)
            t_col = timed(lambda: layer.inverse(z), 1)
        finally:
            cfg.USE_AR_SEQINV = prev
    close(xs, xc, 1e-5, 1e-4)
    close(lds, ldc, LD_RTOL, 5e-4)
    print("poly2048 inverse at 40 rows: seqinv %.2f ms, per-column %.2f ms (%.1fx)"
          % (t_seq * 1e3, t_col * 1e3, t_col / t_seq))
    assert t_seq < t_col
    flush_status_checks()
