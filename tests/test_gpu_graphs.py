"""GPU: graphs.GraphedLogProb, log_prob (nf/models.py:37-40) of a fixed batch
shape replayed as one HIP graph.

* bitwise the eager call on the same rows, for the launch-bound c1 shape
  (2-D two moons, 4-layer RealNVP, H=100: library GEMM conditioners +
  nfk_affine_coupling) and for a chained NSF_CL model (one fused launch);
* new rows copied into the static input give the eager result for them;
* against the CPU oracle at the c1 bench's tolerance;
* after a weight update, ``recapture()`` follows the new weights;
* the reference's data-dependent error (no element inside [-B, B],
  nf/utils.py:63) is raised from the replay's status words.
"""
import os
import sys

import pytest
import torch

import nf.flows as nff
import nf.models as nfm
from normalizingflow_amd import flush_status_checks
from normalizingflow_amd.graphs import GraphedLogProb
from oracle import nf_oracle as orc

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _to(model, D, dev):
    model = model.to(dev)
    model.prior = torch.distributions.MultivariateNormal(torch.zeros(D, device=dev), torch.eye(D, device=dev))
    return model


def test_graphed_c1_bitwise_and_vs_oracle(hip_device):
    import bench
    model, sd, _ = bench.build_model("c1", hip_device)
    g = torch.Generator().manual_seed(0)
    x = bench.moons(4096, generator=g).to(hip_device)
    gl = GraphedLogProb(model, x)
    out = gl().clone()
    ref = model.log_prob(x)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    # new rows through the static input
    x2 = bench.moons(4096, generator=g).to(hip_device)
    out2 = gl(x2).clone()
    assert torch.equal(out2, model.log_prob(x2))
    flush_status_checks()
    lp = orc.model_log_prob(bench.specs_for("c1"), sd, x2.cpu())
    torch.testing.assert_close(out2.cpu(), lp.float(), rtol=1e-5, atol=1e-5)


def _nsf_model(dev, n_layers=4):
    torch.manual_seed(1234)
    flows = [nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[i % 2]) for i in range(n_layers)]
    prior = torch.distributions.MultivariateNormal(torch.zeros(64), torch.eye(64))
    model = nfm.NormalizingFlowModel(prior, flows)
    return _to(model, 64, dev)


def test_graphed_nsf_chain_bitwise_and_recapture(hip_device):
    model = _nsf_model(hip_device)
    g = torch.Generator(device=hip_device).manual_seed(3)
    x = torch.randn(5000, 64, generator=g, device=hip_device)
    gl = GraphedLogProb(model, x)
    assert torch.equal(gl().clone(), model.log_prob(x))
    # a weight update: recaptured by hand
    with torch.no_grad():
        model.flows[1].psi.network[2].weight.mul_(1.5)
    model.invalidate_caches()
    eager = model.log_prob(x)
    assert torch.equal(gl.recapture()().clone(), eager)
    flush_status_checks()


def test_graphed_replay_after_update_and_eager_call(hip_device):
    """a versioned update followed by an eager call (which replaces
    the pack caches) must not leave the graph reading freed packs: the replay
    sees the stale parameter key and recaptures."""
    model = _nsf_model(hip_device)
    x = torch.randn(3000, 64, generator=torch.Generator(device=hip_device).manual_seed(4), device=hip_device)
    gl = GraphedLogProb(model, x)
    before = gl().clone()
    with torch.no_grad():
        model.flows[0].psi.network[0].weight.mul_(0.5)  # bumps the version counter
    eager = model.log_prob(x)                            # new packs replace the cached ones
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    assert gl.stale()
    after = gl().clone()                                 # no recapture() call: replay recaptures
    assert torch.equal(after, eager)
    assert not torch.equal(after, before)
    flush_status_checks()


def test_graphed_stale_after_module_replaced(hip_device):
    """The staleness test (a C++ watch over the module tree's dicts and the
    parameters) sees a replaced layer, not only versioned in-place updates."""
    import copy
    model = _nsf_model(hip_device, n_layers=2)
    x = torch.randn(512, 64, generator=torch.Generator(device=hip_device).manual_seed(6), device=hip_device)
    gl = GraphedLogProb(model, x)
    gl()
    assert not gl.stale()
    model.flows[0] = copy.deepcopy(model.flows[0])
    assert gl.stale()
    eager = model.log_prob(x)
    torch.cuda.synchronize()
    assert torch.equal(gl().clone(), eager)
    assert not gl.stale()
    flush_status_checks()


def test_graphed_keeps_captured_packs_alive(hip_device):
    """Writes through ``p.data`` bump no version: after invalidate_caches() and
    an eager call the graph still replays its capture's weights from the packs
    it holds (not freed allocator memory), until recapture()."""
    model = _nsf_model(hip_device)
    x = torch.randn(3000, 64, generator=torch.Generator(device=hip_device).manual_seed(5), device=hip_device)
    gl = GraphedLogProb(model, x)
    before = gl().clone()
    model.flows[0].psi.network[0].weight.data.mul_(0.5)
    model.invalidate_caches()
    eager = model.log_prob(x)
    # churn the allocator: the freed blocks of unpinned packs would be reused here
    junk = [torch.full((1 << 18,), float("nan"), device=hip_device) for _ in range(64)]
    torch.cuda.synchronize()
    assert not gl.stale()
    assert torch.equal(gl().clone(), before)
    del junk
    assert torch.equal(gl.recapture()().clone(), eager)
    flush_status_checks()


def test_graphed_raises_reference_error_after_replay(hip_device):
    model = _nsf_model(hip_device, n_layers=2)
    x = torch.randn(256, 64, device=hip_device)
    gl = GraphedLogProb(model, x)
    gl()
    flush_status_checks()
    bad = torch.full_like(x, 10.0)  # every element outside [-3, 3]: torch.min of an empty tensor
    with pytest.raises(RuntimeError, match="numel"):  # at the replay (strict) or the flush (deferred)
        gl(bad)
        flush_status_checks()
    with pytest.raises(ValueError):
        gl(torch.zeros(10, 64, device=hip_device))


def test_graphed_sample_consistent_with_eager_kernels(hip_device):
    from normalizingflow_amd.graphs import GraphedSample
    model = _nsf_model(hip_device)
    gs = GraphedSample(model, 3000)
    x1, lp1, z1 = [t.clone() for t in gs()]
    x2, lp2, z2 = [t.clone() for t in gs()]
    assert not torch.equal(z1, z2)  # fresh prior draws per replay
    with torch.no_grad():
        xi, ldi = model.inverse(z2)
    assert torch.equal(x2, xi)
    prior_lp = model.prior.log_prob(z2)
    torch.testing.assert_close(lp2, prior_lp - ldi, rtol=1e-5, atol=1e-4)
    flush_status_checks()


@pytest.mark.parametrize("workload", ["c2", "c3", "c5", "ar", "ar354", "fe162", "poly2048", "rnvp2048"])
def test_graphed_bench_workloads_bitwise(workload, hip_device):
    """bench.py replays log_prob as a graph for per-rank batches <= 2^17 (the
    8-GPU strong-scaling shard, and the applications' 40-row NSF_AR and
    RealNVP-2048 batches): the replay of every bench workload's model is
    bitwise its eager call (c5 at 512 rows: the wide kernel's shape, not its
    batch, is what the graph must carry)."""
    import bench
    model, _, _ = bench.build_model(workload, hip_device)
    D = bench.WORKLOADS[workload][3]
    rows = 512 if workload == "c5" else (40 if workload in ("ar354", "fe162", "poly2048", "rnvp2048") else 3000)
    x = torch.randn(rows, D, generator=torch.Generator(device=hip_device).manual_seed(5), device=hip_device)
    gl = GraphedLogProb(model, x)
    out = gl().clone()
    ref = model.log_prob(x)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    flush_status_checks()
