"""CPU: the host logic of RealNVP's zero-padded halves (flows.RealNVP._fused_half,
rnvp_pad / rnvp_unpad) and the graph wrappers' device checks.  The kernels
themselves run in tests/test_gpu_rnvp_chain.py::test_rnvp_padded_halves_*."""
import pytest
import torch

import nf.flows as nff
from normalizingflow_amd import flows as F_


def test_fused_half_dimension():
    # the kernels take half-dimensions 16, 32, 48, 64: others pad up to the next
    assert F_._rnvp_fused_half(32, 100) == 32
    assert F_._rnvp_fused_half(1, 100) == 16      # c1: D = 2
    assert F_._rnvp_fused_half(20, 100) == 32
    assert F_._rnvp_fused_half(65, 100) is None   # past the kernels: library GEMMs
    assert F_._rnvp_fused_half(5, 140) is None    # H past the kernels
    assert nff.RealNVP(2, hidden_dim=100)._fused_half(100) == 16


def test_pad_unpad_roundtrip():
    x = torch.randn(7, 6)
    xp = F_.rnvp_pad(x, 3, 16)
    assert xp.shape == (7, 32)
    assert torch.equal(xp[:, :3], x[:, :3]) and torch.equal(xp[:, 16:19], x[:, 3:])
    assert not bool(xp[:, 3:16].any()) and not bool(xp[:, 19:].any())
    assert torch.equal(F_.rnvp_unpad(xp, 3, 16), x)
    assert F_.rnvp_pad(x, 3, 3) is x and F_.rnvp_unpad(x, 3, 3) is x


def test_no_fused_pack_off_device():
    # on the CPU the layer reports no fused shape (the kernels would raise)
    layer = nff.RealNVP(2, hidden_dim=100)
    assert layer._fused_pack(torch.device("cpu")) is None
    assert layer._chain_shape(torch.device("cpu")) is None


def test_graph_wrappers_need_a_hip_device():
    from normalizingflow_amd.graphs import GraphedLogProb
    layer = nff.RealNVP(2, hidden_dim=8)
    with pytest.raises(ValueError):
        GraphedLogProb(layer, torch.zeros(4, 2))
