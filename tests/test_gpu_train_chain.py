"""GPU checks of the training forward as one chained launch (config.USE_TRAIN_CHAIN,
models._ChainFn, include/nfk.h nfk_fused_nsf_chain_saved): the train step of
applications/src/train.py:22-28 (loss = -mean(log p(x)), backward) over a run of
fused NSF_CL layers (nf/flows.py:216-253) gives bitwise the loss, z, log|det| and
every gradient of one autograd node and one launch per layer, and the layer
inputs the chain saves are bitwise the per-layer path's.  Against the oracle the
train step is covered by test_gpu_grad.py::test_train_steps_match_oracle, whose
2-layer c3 model now runs through the chain.
"""
import pytest
import torch

import nf.flows as nff
import nf.models as nfm
from normalizingflow_amd import config
from normalizingflow_amd import kernels as K_

pytestmark = pytest.mark.gpu


def _model(n_layers, dev, seed=3):
    torch.manual_seed(seed)
    flows = [nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[i % 2]) for i in range(n_layers)]
    prior = torch.distributions.MultivariateNormal(torch.zeros(64, device=dev), torch.eye(64, device=dev))
    return nfm.NormalizingFlowModel(prior, flows).to(dev)


def _step(model, x, chain, monkeypatch):
    monkeypatch.setattr(config, "USE_TRAIN_CHAIN", chain)
    calls = []
    real = K_.fused_nsf_chain_saved

    def counted(*a, **k):
        calls.append(a[4])  # nlayers
        return real(*a, **k)

    monkeypatch.setattr(K_, "fused_nsf_chain_saved", counted)
    model.zero_grad(set_to_none=True)
    xg = x.clone().requires_grad_(True)
    z, plp, ld = model(xg)
    loss = -torch.mean(plp + ld)
    loss.backward()
    grads = {k: p.grad.clone() for k, p in model.named_parameters()}
    return calls, loss.detach(), z.detach(), ld.detach(), xg.grad.clone(), grads


# (batches of at most a few thousand rows: at >= 32K rows the fused VJP kernel
# itself is not run-to-run reproducible)
@pytest.mark.parametrize("n_layers,rows", [(8, 4097), (3, 1000), (2, 2048)])
def test_train_chain_bitwise_vs_per_layer(n_layers, rows, hip_device, monkeypatch):
    model = _model(n_layers, hip_device)
    x = torch.randn(rows, 64, generator=torch.Generator().manual_seed(rows)).to(hip_device) * 1.2
    calls, *chain = _step(model, x, True, monkeypatch)
    assert calls == [n_layers]  # the whole run was one saved-input chain launch
    calls0, *per_layer = _step(model, x, False, monkeypatch)
    assert calls0 == []
    for a, b, what in zip(chain[:4], per_layer[:4], ("loss", "z", "logdet", "x.grad")):
        assert torch.equal(a, b), what
    for k in chain[4]:
        assert torch.equal(chain[4][k], per_layer[4][k]), k


def test_chain_saves_are_the_layer_inputs(hip_device):
    """The kernel's saved inputs of layers 1.. equal the per-layer forward's
    intermediate x (bitwise), and z and log|det| those of per-layer launches."""
    model = _model(5, hip_device, seed=11)
    run = list(model.flows)
    shape = run[0]._chain_shape(hip_device)
    n_lo, n_up, hidden, K, B = shape
    x = torch.randn(1000, 64, device=hip_device)
    wp, cm = model._chain_args(run, 64, False, x)
    sm = model._chain_save_maps(tuple(run), 64, hip_device)
    z = torch.empty_like(x)
    ld = torch.empty(1000, device=hip_device)
    saves = torch.full((4, 1000, 64), 7.0, device=hip_device)
    with torch.no_grad():
        K_.fused_nsf_chain_saved(x, wp, cm, sm, 5, n_lo, n_up, hidden, z, saves, logdet=ld,
                                 logdet_mode=K_.MODE_WRITE, K=K, tail_bound=B)
        xi, ld_ref = x, torch.zeros(1000, device=hip_device)
        for l, f in enumerate(run):
            if l > 0:
                assert torch.equal(saves[l - 1], xi), l
            xi, ldl = f(xi)
            ld_ref = ld_ref + ldl
    assert torch.equal(z, xi) and torch.equal(ld, ld_ref)


def test_train_chain_raises_like_per_layer(hip_device, monkeypatch):
    """A NaN row under the training chain raises the reference's error (the
    chain's per-layer status words), as the per-layer path does."""
    model = _model(3, hip_device)
    x = torch.randn(512, 64, device=hip_device)
    x[7] = float("nan")
    errs = []
    for chain in (True, False):
        monkeypatch.setattr(config, "USE_TRAIN_CHAIN", chain)
        try:
            xg = x.clone().requires_grad_(True)
            _, plp, ld = model(xg)
            (-torch.mean(plp + ld)).backward()
            errs.append(None)
        except Exception as e:  # the reference's error type, whichever it is
            errs.append((type(e), str(e)))
    assert errs[0] == errs[1]


@pytest.mark.parametrize("width", [60, 68])
def test_train_chain_wrong_width_raises_like_per_layer(width, hip_device, monkeypatch):
    """A batch of the wrong width under the training chain raises the
    per-layer path's error instead of launching the chain kernel on it (which
    would read past x's rows or silently drop columns)."""
    model = _model(3, hip_device)
    x = torch.randn(512, width, device=hip_device)
    errs = []
    for chain in (True, False):
        monkeypatch.setattr(config, "USE_TRAIN_CHAIN", chain)
        with pytest.raises(Exception) as ei:
            xg = x.clone().requires_grad_(True)
            _, plp, ld = model(xg)
            (-torch.mean(plp + ld)).backward()
        errs.append((ei.type, str(ei.value)))
    assert errs[0] == errs[1]
    assert "got %d features" % width in errs[0][1]


@pytest.mark.parametrize("B,D,cols", [(1, 64, list(range(0, 64, 2))), (1000, 64, list(range(1, 64, 2))),
                                      (777, 10, [3, 0, 9]), (5, 8, [])])
def test_gather_cols_ones(B, D, cols, hip_device):
    """nfk_gather_cols_ones (the first Linear's [lower | 1] for its weight and
    bias gradients in one GEMM) is exactly [x[:, cols] | 1]."""
    x = torch.randn(B, D, device=hip_device)
    c = torch.tensor(cols, dtype=torch.int32, device=hip_device)
    got = K_.gather_cols_ones(x, c)
    want = torch.cat([x[:, cols], torch.ones(B, 1, device=hip_device)], 1)
    assert got.shape == (B, len(cols) + 1)
    assert torch.equal(got, want)
