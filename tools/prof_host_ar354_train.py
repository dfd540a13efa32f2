"""Host-side profile (cProfile) of the ar354 train step (NLL fwd + bwd + Adam)
at the applications' 40-row batch."""
import cProfile
import pstats
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

dev = torch.device("cuda", 0)
model, sd, _ = bench.build_model("ar354", dev)
opt = torch.optim.Adam(model.parameters(), lr=1e-4)
x = torch.randn(40, 96, device=dev)


def step():
    opt.zero_grad(set_to_none=True)
    z, plp, ld = model(x)  # train.py:22-25: loss = -mean(prior_lp + log_det)
    loss = -torch.mean(plp + ld)
    loss.backward()
    opt.step()


for _ in range(3):
    step()
torch.cuda.synchronize()
pr = cProfile.Profile()
t = time.perf_counter()
pr.enable()
for _ in range(10):
    step()
pr.disable()
torch.cuda.synchronize()
print("ms per step (profiled)", (time.perf_counter() - t) / 10 * 1e3)
t = time.perf_counter()
for _ in range(10):
    step()
torch.cuda.synchronize()
print("ms per step", (time.perf_counter() - t) / 10 * 1e3)
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
