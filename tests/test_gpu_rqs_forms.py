"""GPU: the two forms of the streaming spline kernel -- k_rqs_coupling (one
round per block) and k_rqs_stream (persistent blocks, register-prefetched
slabs, whole-row z stores, nfk_kernels.hip) -- run the same element math and
the same per-sample log|det| summation order, so they must agree bitwise, on
every parameter mode, direction and map layout (permutation maps take the
whole-row path; maps that leave columns untouched take its scattered
fallback), ragged batches and the per-element log|det| output.  The oracle
parity of the path itself is in test_gpu_parity.py.
"""
import pytest
import torch

from normalizingflow_amd import _lib
from normalizingflow_amd import kernels as K_

pytestmark = pytest.mark.gpu


@pytest.fixture
def form():
    lib = _lib.load()
    prev = lib.nfk_debug_rqs_form(-1)
    yield lib
    lib.nfk_debug_rqs_form(prev)


def _maps(kind, n, dev):
    i32 = dict(dtype=torch.int32, device=dev)
    if kind == "nsf_m1":     # NSF_CL mask [1], dim 2: swap within each particle
        return (torch.arange(0, 2 * n, 2, **i32), torch.arange(1, 2 * n, 2, **i32),
                torch.arange(1, 2 * n, 2, **i32), torch.arange(0, 2 * n, 2, **i32), 2 * n)
    if kind == "prefix":     # lower half first
        return (torch.arange(n, 2 * n, **i32), torch.arange(n, 2 * n, **i32),
                torch.arange(0, n, **i32), torch.arange(0, n, **i32), 2 * n)
    if kind == "partial":    # only some columns touched: scattered fallback
        return (torch.arange(1, 2 * n, 2, **i32), torch.arange(1, 2 * n, 2, **i32), None, None, 2 * n + 4)
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["nsf_m1", "prefix", "partial"])
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("inverse", [False, True])
def test_stream_matches_round_kernel(kind, mode, inverse, form, hip_device):
    dev = hip_device
    n, K, B = 16, 8, 1003                     # ragged: not a multiple of a round
    up_in, up_out, lo_in, lo_out, ncol = _maps(kind, n, dev)
    g = torch.Generator(device=dev).manual_seed(7 + mode)
    x = torch.randn(B, ncol, device=dev, generator=g) * 1.5
    per = 3 * K + 1 if mode == 2 else 3 * K - 1
    params = torch.randn(B, n, per, device=dev, generator=g) * 0.7
    if mode != 0:  # unconstrained_RQS / RQS args: normalised-scale logits are fine as they are
        params = params * 0.5
    outs = []
    for f in (0, 1):
        form.nfk_debug_rqs_form(f)
        z = torch.full((B, ncol), -7.0, device=dev)
        ld = torch.randn(B, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
        lad = torch.zeros(B, n, device=dev)
        st = torch.zeros(1, dtype=torch.int32, device=dev)
        K_.rqs_coupling(x, params, up_in, up_out, z, lo_in=lo_in, lo_out=lo_out, logdet=ld, logdet_mode=2,
                        lad_out=lad, K=K, left=-3.0, right=3.0, bottom=-3.0, top=3.0, param_mode=mode,
                        inverse=inverse, status=st)
        torch.cuda.synchronize()
        outs.append((z.cpu(), ld.cpu(), lad.cpu(), st.cpu()))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    if kind == "partial":  # untouched columns keep z's previous contents
        untouched = torch.ones(ncol, dtype=torch.bool)
        untouched[up_out.cpu().long()] = False
        assert torch.all(outs[1][0][:, untouched] == -7.0)
