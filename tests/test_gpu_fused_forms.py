"""GPU parity of the 16-coordinate fused NSF kernel (k_fused_nsf in
nfk_fused_impl.h) in both of its forms -- whole records (two workgroups per
CU) and the split form (records cut into sub-records of NS tiles, three
workgroups per CU) -- over the hidden widths (KBH = 1..4, with and without the
f32 tail step), K, mask and chunk counts it accepts, forward and inverse,
against the CPU oracle (nf/flows.py:216-253, nf/utils.py:27-152).

Tolerances as tests/test_gpu_wide.py: z rtol 1e-5 / atol 5e-5; per-layer
log|det| rtol 1e-5 / atol 3e-4.  The two forms run the same arithmetic in
the same order, so they also agree bitwise.
"""
import pytest
import torch

import nf.flows as nff
from normalizingflow_amd import _lib
from normalizingflow_amd import kernels as K_
from oracle import nf_oracle as orc

pytestmark = pytest.mark.gpu

Z_RTOL, Z_ATOL = 1e-5, 5e-5
LD_RTOL, LD_ATOL = 1e-5, 3e-4

# (size, dim, K, hidden, mask)
SHAPES = [
    (32, 2, 8, 100, [1]),   # c3 layer: KBH 3 + f32 tail, two chunks
    (32, 2, 8, 100, [0]),
    (16, 2, 4, 64, [0]),    # KBH 2, one chunk
    (12, 2, 5, 33, [1]),    # KBH 1 + tail, partial chunk
    (20, 2, 6, 128, [0]),   # KBH 4 (2-tile sub-records)
    (24, 2, 10, 130, [1]),  # KBH 4 + tail, K 10
    (30, 3, 8, 100, [1]),   # dim 3: 30 lower / 60 upper coordinates, four chunks
    (40, 2, 8, 100, [1]),   # two layer-1 k-blocks (layer-1 record larger than a sub-record)
]


def _ids(s):
    return "s%d_d%d_k%d_h%d_m%s" % (s[0], s[1], s[2], s[3], "".join(map(str, s[4])))


@pytest.fixture
def form():
    lib = _lib.load()
    prev = lib.nfk_debug_fused_form(-1)
    yield lib
    lib.nfk_debug_fused_form(prev)


def _run(layer, x, inverse):
    with torch.no_grad():
        z, ld = (layer.inverse(x) if inverse else layer(x))
    assert layer._pack_cache is not None  # the fused kernel ran
    return z.cpu(), ld.cpu()


@pytest.mark.parametrize("shape", SHAPES, ids=_ids)
@pytest.mark.parametrize("inverse", [False, True])
def test_fused_forms_vs_oracle(shape, inverse, form, hip_device):
    size, dim, K, hidden, mask = shape
    n_lo, n_up = len(mask) * size, (dim - len(mask)) * size
    assert K_.fused_nsf_supported(n_lo, n_up, hidden, K)
    torch.manual_seed(size + 7 * K + hidden)
    layer = nff.NSF_CL(size=size, dim=dim, K=K, B=3, hidden_dim=hidden, mask=mask)
    x = torch.randn(1000, size * dim, generator=torch.Generator().manual_seed(3)) * 1.3
    sd = {k: v.detach().cpu() for k, v in layer.state_dict().items()}
    z_ref, ld_ref = orc.nsf_cl(x, sd, "", size, dim, K, 3, mask, inverse=inverse)
    dev = layer.to(hip_device)
    xd = x.to(hip_device)
    out = {}
    for f in (0, 1):
        form.nfk_debug_fused_form(f)
        out[f] = _run(dev, xd, inverse)
        torch.testing.assert_close(out[f][0], z_ref, rtol=Z_RTOL, atol=Z_ATOL)
        torch.testing.assert_close(out[f][1], ld_ref, rtol=LD_RTOL, atol=LD_ATOL)
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
