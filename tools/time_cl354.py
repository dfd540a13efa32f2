"""Time the applications' NSF_CL branch (setup.py:59-62 at Einstein.yaml's sizes:
32 particles x 3 dims, K 32, H 354, six-mask cycle) log_prob at a few batches."""
import sys
import time

import torch

sys.path.insert(0, ".")
import nf.flows as nff  # noqa: E402
import nf.models as nfm  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
B = (32 / (8 * 1.28)) ** (1.0 / 3.0)
masks = [[0], [1], [2], [0, 1], [1, 2], [0, 2]]
flows = [nff.NSF_CL(size=32, dim=3, K=32, B=B, hidden_dim=354, mask=m) for m in masks]
prior = torch.distributions.MultivariateNormal(torch.zeros(96, device=dev), torch.eye(96, device=dev))
model = nfm.NormalizingFlowModel(prior, flows).to(dev)
model.prior = prior
for rows in (40, 4096, 65536):
    x = torch.randn(rows, 96, device=dev) * 0.6
    with torch.no_grad():
        for _ in range(3):
            model.log_prob(x)
        torch.cuda.synchronize()
        n = 20
        t = time.perf_counter()
        for _ in range(n):
            model.log_prob(x)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / n
    print("cl354 rows %6d: %.3f ms per 6-layer log_prob, %.3g samples/s" % (rows, dt * 1e3, rows / dt))
