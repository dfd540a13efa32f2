"""Sample-sharded data parallelism over the GPUs of one node.

Every layer in scope is independent per sample, so the
batch is split by rows across ranks (one process per GPU, backend "nccl" =
RCCL over xGMI) with replicated weights and no collective on the data path.
The only exchanges are the ones the path really has:

  * the NLL of training / evaluation (applications/src/train.py:22-25):
    one all_reduce(SUM) of [sum log p, count] -- 16 bytes per step;
  * Radial's batch-global norm (nf/flows_1.py:90): one all_reduce(SUM) of the
    fp64 squared norm before its elementwise step (``attach_process_group``);
  * training (train.py:22-28 run data-parallel): the parameter gradients,
    averaged by DistributedDataParallel's bucketed all_reduce, overlapped with
    the backward (``data_parallel``), of the per-rank loss ``sharded_nll``
    (exact for uneven shards).  The c3 model has 8 x 0.55 M fp32
    parameters = 17.6 MB of gradient per step, one or two 25 MB buckets.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .flows import Radial

__all__ = ["shard_range", "shard", "nll_allreduce", "sharded_nll", "attach_process_group",
           "init_from_env", "data_parallel"]


def shard_range(n, rank, world):
    """Rows [lo, hi) of an n-row batch owned by ``rank`` (contiguous, balanced)."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shard(x, rank=None, world=None):
    """This rank's contiguous row slice of a replicated batch."""
    rank = dist.get_rank() if rank is None else rank
    world = dist.get_world_size() if world is None else world
    lo, hi = shard_range(x.shape[0], rank, world)
    return x[lo:hi]


def nll_allreduce(log_prob, group=None):
    """Global mean negative log-likelihood, -mean(log p) over all ranks'
    samples (train.py:23-25).  Reduces [sum, count] in fp64: 16 bytes."""
    acc = torch.stack([log_prob.double().sum(),
                       torch.tensor(float(log_prob.numel()), dtype=torch.float64,
                                    device=log_prob.device)])
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(acc, op=dist.ReduceOp.SUM, group=group)
    return (-(acc[0] / acc[1])).to(log_prob.dtype)


def sharded_nll(log_prob, n_global=None, group=None):
    """This rank's training loss for ``data_parallel``: -sum(log p) * world / N
    over its rows, N the global row count (all-reduced from the shards when
    not given).  DistributedDataParallel averages the gradients over the
    world, so the averaged gradient is exactly that of the global
    -mean(log p) (train.py:23-27) for ANY split of the rows -- averaging per
    rank means (-mean of each shard) is that only when the shards are equal.
    The mean over ranks of the returned values is the global NLL.

    Pass ``n_global`` in a training loop (the caller knows it: the sum of
    shard_range's sizes): without it every call adds a count all-reduce,
    kept on the device (no host sync) but still one collective per step."""
    world = 1
    if dist.is_available() and dist.is_initialized():
        world = dist.get_world_size(group)
        if n_global is None:
            cnt = torch.tensor([float(log_prob.numel())], dtype=torch.float64, device=log_prob.device)
            dist.all_reduce(cnt, op=dist.ReduceOp.SUM, group=group)
            return -log_prob.sum() * (world / cnt[0]).to(log_prob.dtype)
    if n_global is None:
        n_global = log_prob.numel()
    return -log_prob.sum() * (world / float(n_global))


def attach_process_group(model, group=None):
    """Make batch-global layers (Radial) reduce over ``group`` -- call once per
    model when the batch is sharded; other layers need nothing."""
    g = group if group is not None else dist.group.WORLD
    for m in model.modules():
        if isinstance(m, Radial):
            m.process_group = g
    return model


def init_from_env(backend=None, force=False):
    """torchrun-style init: RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* from env.
    Returns (rank, world, local_rank); a no-op single process when WORLD_SIZE
    is unset, unless ``force`` (a world of one still gets a process group, so
    the collectives run through the backend, e.g. RCCL on a one-GPU box)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if (world > 1 or force) and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


def data_parallel(model, device=None, bucket_cap_mb=25, **kw):
    """Wrap a model for sample-sharded training: batch-global layers get the
    process group, then DistributedDataParallel averages the gradients across
    ranks.  Each rank feeds its own rows (``shard``) and minimises
    ``sharded_nll`` of its rows, whose averaged gradient is the gradient of
    the global mean NLL (train.py:23-27) for equal and unequal shards alike."""
    from torch.nn.parallel import DistributedDataParallel as DDP
    attach_process_group(model)
    ids = None
    if device is not None and torch.device(device).type == "cuda":
        ids = [torch.device(device).index or 0]
    return DDP(model, device_ids=ids, bucket_cap_mb=bucket_cap_mb, **kw)
