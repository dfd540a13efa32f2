"""CPU: the bench's synthetic data: the c1 two-moons rows are
seeded, shaped and placed like the make_moons formula; the other workloads
draw x ~ N(0, I)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_moons_shape_seed_and_arcs():
    a = bench.moons(4096, generator=torch.Generator().manual_seed(0))
    b = bench.moons(4096, generator=torch.Generator().manual_seed(0))
    assert a.shape == (4096, 2) and a.dtype == torch.float32
    assert torch.equal(a, b)
    # noise-free points lie on the two unit half circles centred (0, 0) and (1, 0.5)
    c = bench.moons(1001, noise=0.0, generator=torch.Generator().manual_seed(1)).double()
    r_out = (c - torch.tensor([0.0, 0.0], dtype=torch.float64)).norm(dim=1)
    r_in = (c - torch.tensor([1.0, 0.5], dtype=torch.float64)).norm(dim=1)
    on_out = (r_out - 1).abs() < 1e-6
    on_in = (r_in - 1).abs() < 1e-6
    assert bool((on_out | on_in).all())
    assert int(on_out.sum()) == 500 and int((on_in & ~on_out).sum()) == 501
    assert bool((c[on_out, 1] >= -1e-6).all()) and bool((c[on_in & ~on_out, 1] <= 0.5 + 1e-6).all())


def test_make_x_per_workload():
    g = torch.Generator().manual_seed(0)
    assert bench.make_x("c1", 64, g, "cpu").shape == (64, 2)
    assert bench.make_x("c3", 64, g, "cpu").shape == (64, 64)
    assert bench.make_x("c5", 8, g, "cpu").shape == (8, 256)
    assert bench.DEFAULT_BATCH.get("c1") == 4096
