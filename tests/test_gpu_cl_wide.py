"""GPU: NSF_CL layers with the applications' wide conditioner (setup.py:59-62:
32 particles x 3 dims, nsplines 32, hidden 354) on the fused kernel
k_fused_cl (nfk_fused_ar.hip, reached through nfk_fused_nsf_*): one launch per
layer, layers 1-2 of the FCNN once per sample, the output layer streamed as
one record per upper coordinate with its spline (nf/flows.py:216-253).

Checked against the CPU oracle and the unfused path (library GEMMs +
nfk_rqs_coupling) at every mask of the applications' six-mask cycle, both
directions, ragged batches; log|det| accumulate mode; the no-element-inside
error; per-sample independence (an outlier row leaves every other row's
output bitwise unchanged)."""
import pytest
import torch

import nf.flows as nff
from normalizingflow_amd import config, flush_status_checks
from normalizingflow_amd import kernels as K_
from oracle import nf_oracle as orc

pytestmark = pytest.mark.gpu

B_APP = (32 / (8 * 1.28)) ** (1.0 / 3.0)
MASKS = ([0], [1], [2], [0, 1], [1, 2], [0, 2])
Z_RTOL, Z_ATOL = 1e-5, 2e-5
LD_RTOL, LD_ATOL = 1e-5, 2e-4  # log|det| sums 32-64 coordinates


def close(a, b, rtol, atol):
    torch.testing.assert_close(a.detach().cpu(), b.detach().cpu(), rtol=rtol, atol=atol)


def _layer(mask, seed=3):
    torch.manual_seed(seed)
    return nff.NSF_CL(size=32, dim=3, K=32, B=B_APP, hidden_dim=354, mask=mask)


def _sd(layer):
    return {k: v.detach().cpu() for k, v in layer.state_dict().items()}


def _unfused(layer, x, inverse):
    prev = config.USE_FUSED
    config.USE_FUSED = False
    try:
        layer.invalidate_caches()
        return layer.inverse(x) if inverse else layer(x)
    finally:
        config.USE_FUSED = prev
        layer.invalidate_caches()


@pytest.mark.parametrize("mask", MASKS)
@pytest.mark.parametrize("inverse", [False, True])
def test_cl_wide_vs_oracle_and_unfused(mask, inverse, hip_device):
    layer = _layer(mask)
    n_lo, n_up = 32 * len(mask), 32 * (3 - len(mask))
    assert K_.fused_nsf_supported(n_lo, n_up, 354, 32)
    assert K_.fused_nsf_chain_max(n_lo, n_up, 354, 32) == 0  # one launch per layer
    sd = _sd(layer)
    x = torch.randn(333, 96, generator=torch.Generator().manual_seed(len(mask) * 7 + inverse)) * 0.7
    with torch.no_grad():
        z_ref, ld_ref = orc.nsf_cl(x, sd, "", 32, 3, 32, B_APP, mask, inverse=inverse)
    layer = layer.to(hip_device)
    xd = x.to(hip_device)
    with torch.no_grad():
        assert layer._fused_pack(xd.device) is not None
        z, ld = layer.inverse(xd) if inverse else layer(xd)
        zu, ldu = _unfused(layer, xd, inverse)
    close(z, z_ref, Z_RTOL, Z_ATOL)
    close(ld, ld_ref, LD_RTOL, LD_ATOL)
    close(z, zu, Z_RTOL, Z_ATOL)
    close(ld, ldu, LD_RTOL, LD_ATOL)
    flush_status_checks()


def test_cl_wide_round_trip_and_modes(hip_device):
    """inverse(forward(x)) = x, the two log|det| cancel (a prefix mask: the
    reference's inverse reads the lower coordinates at the mask positions of
    its input, which the masked-first forward output holds only for prefix
    masks); the kernel's accumulate mode adds to the buffer; 1, 65, 4,096 rows."""
    layer = _layer([0, 1], seed=5).to(hip_device)
    for rows in (1, 65, 4096):
        x = torch.randn(rows, 96, device=hip_device) * 0.5
        with torch.no_grad():
            z, ld = layer(x)
            xr, ldr = layer.inverse(z)
        assert float((xr - x).abs().max()) < 1e-4
        assert float((ld + ldr).abs().max()) < 1e-3
    maps = layer._maps(x.device)
    pack = layer._fused_pack(x.device)
    z1 = torch.empty_like(x)
    ld1 = torch.zeros(x.shape[0], device=hip_device)
    K_.fused_nsf(x, pack, maps.up_in, maps.up_out, maps.lo_in, maps.lo_out, 354, z1, logdet=ld1,
                 logdet_mode=K_.MODE_WRITE, K=32, tail_bound=B_APP)
    ld2 = torch.full((x.shape[0],), 2.5, device=hip_device)
    z2 = torch.empty_like(x)
    K_.fused_nsf(x, pack, maps.up_in, maps.up_out, maps.lo_in, maps.lo_out, 354, z2, logdet=ld2,
                 logdet_mode=K_.MODE_ACC, K=32, tail_bound=B_APP)
    assert torch.equal(z1, z2)
    assert torch.equal(ld2, ld1 + 2.5)
    flush_status_checks()


def test_cl_wide_no_element_inside_raises(hip_device):
    layer = _layer([1], seed=7).to(hip_device)
    x = torch.full((300, 96), 10.0, device=hip_device)
    prev = config.STRICT_CHECKS
    config.STRICT_CHECKS = True
    try:
        with torch.no_grad(), pytest.raises(RuntimeError, match="numel"):
            layer(x)
    finally:
        config.STRICT_CHECKS = prev


def test_cl_wide_outlier_rows_bitwise(hip_device):
    """Per-sample layer-1 scaling: rows holding 1e8 / inf / NaN leave every
    other row's z and log|det| bitwise unchanged."""
    layer = _layer([0], seed=9).to(hip_device)
    x = torch.randn(200, 96, device=hip_device) * 0.6
    xo = x.clone()
    rows = [3, 21, 40, 77]
    for r, v in zip(rows, (1e8, float("inf"), float("nan"), -1e4)):
        xo[r] = v
    keep = torch.ones(200, dtype=torch.bool, device=hip_device)
    keep[rows] = False
    with torch.no_grad():
        z, ld = layer(x)
        zo, ldo = layer(xo)
    assert torch.equal(z[keep], zo[keep])
    assert torch.equal(ld[keep], ldo[keep])


@pytest.mark.parametrize("rows", [1, 40, 333, 4096])
@pytest.mark.parametrize("inverse", [False, True])
def test_cl_wide_coordinate_split_bitwise(rows, inverse, hip_device):
    """Small batches split the upper coordinates over workgroups
    (nfk_fused_nsf_ws + the per-coordinate log|det| workspace): z, log|det|
    (modes 1 and 2) and the status word are bitwise the unsplit launch's."""
    layer = _layer([1], seed=11).to(hip_device)
    x = torch.randn(rows, 96, device=hip_device) * 0.6
    maps = layer._maps(x.device)
    pack = layer._fused_pack(x.device)
    n_lo, n_up = maps.lo_in.numel(), maps.up_in.numel()
    nws = K_._lib.load().nfk_fused_nsf_workspace(n_lo, n_up, 354, 32, rows, int(inverse))
    if rows <= 333:
        assert nws == n_up * rows
    res = []
    for split in (False, True):
        out = []
        for mode, init in ((K_.MODE_WRITE, 0.0), (K_.MODE_ACC, 1.5)):
            z = torch.empty_like(x)
            ld = torch.full((rows,), init, device=hip_device)
            st = torch.zeros(1, dtype=torch.int32, device=hip_device)
            if split:
                K_.fused_nsf(x, pack, maps.up_in, maps.up_out, maps.lo_in, maps.lo_out, 354, z, logdet=ld,
                             logdet_mode=mode, K=32, tail_bound=B_APP, inverse=inverse, status=st)
            else:
                K_._lib.call("nfk_fused_nsf", x.data_ptr(), 96, pack.data_ptr(), maps.up_in.data_ptr(),
                             maps.up_out.data_ptr(), n_up, maps.lo_in.data_ptr(), maps.lo_out.data_ptr(), n_lo,
                             354, z.data_ptr(), 96, ld.data_ptr(), mode, rows, 32, float(B_APP), int(inverse),
                             st.data_ptr(), K_._stream(x.device))
            out += [z, ld, st]
        torch.cuda.synchronize()
        res.append(out)
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("mask", [[0], [1, 2]])
@pytest.mark.parametrize("inverse", [False, True])
def test_cl_config_defaults_vs_oracle(mask, inverse, hip_device):
    """The applications' config.py defaults for the NSF_CL branch (nsplines 32,
    hidden 100) on the same kernel (k_fused_cl's H = 100 instance): vs the
    oracle and the unfused path, 1 and 333 rows."""
    torch.manual_seed(17 + len(mask))
    layer = nff.NSF_CL(size=32, dim=3, K=32, B=B_APP, hidden_dim=100, mask=mask)
    n_lo, n_up = 32 * len(mask), 32 * (3 - len(mask))
    assert K_.fused_nsf_supported(n_lo, n_up, 100, 32)
    sd = _sd(layer)
    layer = layer.to(hip_device)
    for rows in (1, 333):
        x = torch.randn(rows, 96, generator=torch.Generator().manual_seed(rows)) * 0.7
        xd = x.to(hip_device)
        with torch.no_grad():
            assert layer._fused_pack(xd.device) is not None
            z, ld = layer.inverse(xd) if inverse else layer(xd)
            zu, ldu = _unfused(layer, xd, inverse)
            if rows > 1:
                z_ref, ld_ref = orc.nsf_cl(x, sd, "", 32, 3, 32, B_APP, mask, inverse=inverse)
                close(z, z_ref, Z_RTOL, Z_ATOL)
                close(ld, ld_ref, LD_RTOL, LD_ATOL)
        close(z, zu, Z_RTOL, Z_ATOL)
        close(ld, ldu, LD_RTOL, LD_ATOL)
    flush_status_checks()
