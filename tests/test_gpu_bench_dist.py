"""GPU: bench.py's own N = 2 data path, end to end (BASELINE c4 / the north
star's strong scaling).  torchrun starts two ranks of
bench.py on the box's one device over gloo (the driver's 8-GPU run uses the
same code over RCCL).  Each rank runs the full 8-layer c3 model on its shard
and the step ends in the NLL all-reduce (applications/src/train.py:23-25);
the reported NLL must equal the CPU oracle's -mean(log_prob) over the same
rows (nf/models.py:37-40) within the north star's 1e-5 relative."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _nll_ref(hip_device, sizes):
    """The oracle's -mean(log_prob) over the rows the ranks benched: rank r
    draws its rows from a device generator seeded by r."""
    import bench
    from oracle import nf_oracle as orc
    xs = []
    for rank, n in enumerate(sizes):
        g = torch.Generator(device=hip_device).manual_seed(rank)
        xs.append(torch.randn(n, 64, generator=g, device=hip_device).cpu())
    x = torch.cat(xs)
    _, sd, _ = bench.build_model("c3", hip_device)
    ref = orc.model_log_prob(bench.specs_for("c3"), {k: v.cpu() for k, v in sd.items()}, x)
    return float(-ref.double().mean())


def _bench_world2(extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo",
           "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--parity-rows", "1024", *extra]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_world2_weak_and_strong_nll_vs_oracle(hip_device):
    """The driver's N > 1 invocation (no --scaling): ONE line with the weak
    loop (c4: --batch rows per rank) as its value and the strong loop (the
    metric's global batch split over the ranks) as its "strong" object, each
    NLL equal to the oracle's over the rows it ran."""
    sys.path.insert(0, REPO)
    from normalizingflow_amd.dist import shard_range
    weak_rows, strong_rows = 12288, 32769  # the strong batch does not divide by 2: shards 16385 / 16384
    line = _bench_world2(["--batch", str(weak_rows), "--global-batch", str(strong_rows)])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["global_batch"] == 2 * weak_rows and line["config"]["backend"] == "gloo"
    assert line["value"] > 0 and line["parity"]["pass"]
    st = line["strong"]
    assert st["scaling"] == "strong" and st["global_batch"] == strong_rows and st["per_gpu_batch"] == 16385
    assert st["value"] > 0 and st["ms_per_step"] > 0 and st["parity"]["pass"]
    ref_w = _nll_ref(hip_device, [weak_rows, weak_rows])
    assert abs(line["nll"] - ref_w) <= 1e-5 * abs(ref_w), (line["nll"], ref_w)
    sizes = [hi - lo for lo, hi in (shard_range(strong_rows, r, 2) for r in range(2))]
    ref_s = _nll_ref(hip_device, sizes)
    assert abs(st["nll"] - ref_s) <= 1e-5 * abs(ref_s), (st["nll"], ref_s)


@pytest.mark.parametrize("scaling,rows", [("strong", 32768), ("weak", 12288)])
def test_bench_world2_single_mode_nll_vs_oracle(hip_device, scaling, rows):
    sys.path.insert(0, REPO)
    from normalizingflow_amd.dist import shard_range
    size_arg = ["--global-batch", str(rows)] if scaling == "strong" else ["--batch", str(rows)]
    line = _bench_world2(["--scaling", scaling, *size_arg])
    total = rows if scaling == "strong" else 2 * rows
    assert line["n_gpus"] == 2 and line["scaling"] == scaling and "strong" not in line
    assert line["config"]["global_batch"] == total and line["config"]["backend"] == "gloo"
    assert line["value"] > 0 and line["parity"]["pass"]
    sizes = [(hi - lo) if scaling == "strong" else rows for lo, hi in (shard_range(rows, r, 2) for r in range(2))]
    ref = _nll_ref(hip_device, sizes)
    assert abs(line["nll"] - ref) <= 1e-5 * abs(ref), (line["nll"], ref)


def test_bench_gpus2_without_launcher_spawns_ranks(hip_device):
    """`python bench.py --gpus 2` with no launcher (WORLD_SIZE unset) starts its
    own two ranks (bench.spawn_ranks, torchrun's environment contract): ONE
    line with n_gpus 2 whose all-reduced NLL equals the oracle's over both
    ranks' rows -- however the driver invokes the N-GPU run, it measures N ranks."""
    rows = 12288
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo",
           "--scaling", "weak", "--batch", str(rows), "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--parity-rows", "1024"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 2 * rows
    assert line["config"]["backend"] == "gloo" and line["parity"]["pass"]
    ref = _nll_ref(hip_device, [rows, rows])
    assert abs(line["nll"] - ref) <= 1e-5 * abs(ref), (line["nll"], ref)


def test_bench_rccl_world1_nll_vs_oracle(hip_device):
    """The RCCL leg of the same path: one rank under torchrun with a real
    "nccl" (RCCL) process group (--dist keeps the group and the NLL
    all-reduce at N = 1), so the collective the driver's 8-GPU run uses
    executes on the hardware; the all-reduced NLL equals the oracle's."""
    sys.path.insert(0, REPO)
    import bench
    from oracle import nf_oracle as orc

    rows = 8192
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "1", "--backend", "nccl", "--dist",
           "--batch", str(rows), "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
           "--parity-rows", "1024"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["config"]["backend"] == "nccl"
    assert line["value"] > 0 and line["parity"]["pass"] and line["nll"] is not None

    g = torch.Generator(device=hip_device).manual_seed(0)
    x = torch.randn(rows, 64, generator=g, device=hip_device).cpu()
    _, sd, _ = bench.build_model("c3", hip_device)
    ref = orc.model_log_prob(bench.specs_for("c3"), {k: v.cpu() for k, v in sd.items()}, x)
    nll_ref = float(-ref.double().mean())
    assert abs(line["nll"] - nll_ref) <= 1e-5 * abs(nll_ref), (line["nll"], nll_ref)


def test_bench_c1_moons_vs_oracle(hip_device):
    """BASELINE c1 (2-D two moons, 4-layer RealNVP, H=100, B=4096) through
    bench.py on the GPU: the benched log_prob of every row vs the oracle."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--workload", "c1", "--steps", "5",
           "--warmup", "2", "--no-cpu-baseline", "--parity-rows", "4096"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["config"]["global_batch"] == 4096 and line["value"] > 0
    assert line["parity"]["rows"] == 4096 and line["parity"]["pass"], line["parity"]
