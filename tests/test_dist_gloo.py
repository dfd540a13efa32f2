"""Multi-process (gloo, world_size 2) checks of the sample-sharded data path:
row sharding covers the batch exactly once, the NLL all-reduce equals the
single-process -mean(log p), and batch-global layers get the process group.
The HIP kernels are not called (no GPU here); bench.py's N>1 path uses the
same helpers over RCCL."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        from normalizingflow_amd import dist as nfd
        import nf.flows as nff
        r, w, _ = nfd.init_from_env(backend="gloo")
        assert (r, w) == (rank, world) and dist.is_initialized()
        g = torch.Generator().manual_seed(0)
        full = torch.randn(1001, 3, generator=g)
        lp_full = full.sum(1)
        mine = nfd.shard(lp_full)
        lo, hi = nfd.shard_range(1001, rank, world)
        nll = nfd.nll_allreduce(mine)
        # gather row ranges to check coverage
        rng = torch.tensor([lo, hi], dtype=torch.int64)
        allr = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allr, rng)
        model = torch.nn.ModuleList([nff.Radial(3), nff.Planar(3)])
        nfd.attach_process_group(model)
        q.put((rank, float(nll), float(-lp_full.mean()), [t.tolist() for t in allr],
               model[0].process_group is not None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface failures to the parent
        q.put((rank, repr(e)))


def test_sharded_nll_allreduce_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
    for o in out:
        assert len(o) == 5, o
        rank, nll, ref, ranges, has_pg = o
        assert abs(nll - ref) < 1e-5
        assert has_pg
        covered = sorted(tuple(r) for r in ranges)
        assert covered[0][0] == 0 and covered[-1][1] == 1001
        assert all(a[1] == b[0] for a, b in zip(covered, covered[1:]))


@pytest.mark.parametrize("n,world", [(10, 3), (7, 8), (1 << 20, 8), (0, 2)])
def test_shard_range_partitions(n, world):
    from normalizingflow_amd.dist import shard_range
    spans = [shard_range(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1


# --------------------------------------------------------------------------- DDP, uneven shards
class _OracleModel(torch.nn.Module):
    """The oracle's differentiable c3-style model (CPU) as a module, so DDP
    can average its gradients; the HIP path needs a GPU (tests/test_gpu_grad.py
    runs the same check through the kernels)."""

    def __init__(self, sd, specs):
        super().__init__()
        self.names = list(sd)
        self.params = torch.nn.ParameterList([torch.nn.Parameter(sd[k].clone()) for k in self.names])
        self.specs = specs

    def forward(self, x):
        from oracle import nf_oracle as orc
        sd = dict(zip(self.names, self.params))
        _, plp, ld = orc.model_forward(self.specs, sd, x)
        return plp + ld


def _small_sd():
    import nf.flows as nff
    import nf.models as nfm
    torch.manual_seed(5)
    flows = [nff.NSF_CL(size=4, dim=2, K=4, B=3, hidden_dim=16, mask=[i % 2]) for i in range(2)]
    m = nfm.NormalizingFlowModel(torch.distributions.MultivariateNormal(torch.zeros(8), torch.eye(8)), flows)
    return {k: v.detach().clone() for k, v in m.state_dict().items()}


def _ddp_worker(rank, world, port, x, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    try:
        torch.set_num_threads(1)
        from normalizingflow_amd import dist as nfd
        from oracle import nf_oracle as orc
        nfd.init_from_env(backend="gloo")
        model = _OracleModel(_small_sd(), orc.nsf_cl_specs(2, 4, 2, 4, 3, [[0], [1]]))
        ddp = nfd.data_parallel(model)
        lp = ddp(nfd.shard(x))
        loss = nfd.sharded_nll(lp)
        loss.backward()
        vals = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(vals, loss.detach().double().reshape(1))
        q.put((rank, {k: p.grad.numpy().copy() for k, p in zip(model.names, model.params)},
               float(sum(v.item() for v in vals) / world), int(lp.numel())))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        q.put((rank, traceback.format_exc() + repr(e)))


def test_ddp_uneven_shards_grad_equals_full_batch_world3():
    """3 ranks on 100 rows (shards 34/33/33): the DDP-averaged
    gradient of dist.sharded_nll equals the full-batch gradient of
    -mean(log p) (train.py:23-27) at 1e-6, and the mean of the rank losses is
    the global NLL."""
    from oracle import nf_oracle as orc
    torch.set_num_threads(2)
    sd = _small_sd()
    x = torch.randn(100, 8, generator=torch.Generator().manual_seed(11)) * 0.8
    ref = _OracleModel(sd, orc.nsf_cl_specs(2, 4, 2, 4, 3, [[0], [1]]))
    lp = ref(x)
    nll = -lp.mean()
    nll.backward()
    nll_v = float(nll.detach())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_ddp_worker, args=(r, 3, port, x, q)) for r in range(3)]
    for p in ps:
        p.start()
    out = [q.get(timeout=180) for _ in range(3)]
    for p in ps:
        p.join(timeout=60)
    assert sorted(o[3] for o in out if len(o) == 4) == [33, 33, 34], out
    for o in out:
        assert len(o) == 4, o
        rank, grads, mean_loss, n = o
        assert abs(mean_loss - nll_v) <= 1e-6 * abs(nll_v)
        for k, p in zip(ref.names, ref.params):
            g = torch.from_numpy(grads[k])
            err = float((g - p.grad).abs().max())
            assert err <= 1e-6 * max(float(p.grad.abs().max()), 1e-12), (rank, k, err)
