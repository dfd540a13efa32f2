"""Sharded data path on the GPU, world_size 2 (gloo over CUDA tensors, both
ranks on the box's one device): a batch-global Radial layer (flows_1.py:90)
whose squared norm is all-reduced across shards must equal the unsharded
oracle, and the sharded c3 NLL must equal the single-process NLL."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, x, sd_radial, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    try:
        import torch.distributed as dist
        from normalizingflow_amd import dist as nfd
        import nf.flows as nff
        import nf.models as nfm
        nfd.init_from_env(backend="gloo")
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        lo, hi = nfd.shard_range(x.shape[0], rank, world)
        layer = nff.Radial(x.shape[1])
        layer.load_state_dict(sd_radial)
        layer = layer.to(dev)
        nfd.attach_process_group(torch.nn.ModuleList([layer]))
        with torch.no_grad():
            z, ld = layer(x[lo:hi].to(dev))
        # c3-shaped 2-layer NSF_CL model, same weights on every rank
        torch.manual_seed(1234)
        flows = [nff.NSF_CL(size=32, dim=2, K=8, B=3, hidden_dim=100, mask=[i % 2]) for i in range(2)]
        prior = torch.distributions.MultivariateNormal(torch.zeros(64, device=dev),
                                                       torch.eye(64, device=dev))
        model = nfm.NormalizingFlowModel(prior, flows).to(dev)
        g = torch.Generator().manual_seed(5)
        xb = torch.randn(3001, 64, generator=g)
        a, b = nfd.shard_range(xb.shape[0], rank, world)
        nll = nfd.nll_allreduce(model.log_prob(xb[a:b].to(dev)))
        full = float(-model.log_prob(xb.to(dev)).double().mean())
        q.put((rank, lo, z.cpu().numpy(), ld.cpu().numpy(), float(nll), full))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, repr(e)))


def test_sharded_radial_and_nll_world2():
    from oracle import nf_oracle as orc
    import nf.flows as nff
    torch.manual_seed(3)
    ref_layer = nff.Radial(16)
    ref_layer.reset_parameters(16)
    sd = {k: v.detach().clone() for k, v in ref_layer.state_dict().items()}
    x = torch.randn(4099, 16)
    z_ref, ld_ref = orc.radial(x, sd, "")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, x, sd, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = [q.get(timeout=300) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
    for o in out:
        assert len(o) == 6, o
    out.sort(key=lambda o: o[1])
    z = torch.cat([torch.from_numpy(o[2]) for o in out])
    torch.testing.assert_close(z, z_ref, rtol=1e-5, atol=2e-5)
    for o in out:
        torch.testing.assert_close(torch.from_numpy(o[3]), ld_ref, rtol=1e-5, atol=5e-5)
        assert abs(o[4] - o[5]) < 1e-5 * abs(o[5]) + 1e-6
