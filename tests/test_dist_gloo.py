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
