"""Host-side profile (cProfile) of the ar354 log_prob step at the applications'
40-row batch: where the time between kernel launches goes."""
import cProfile
import pstats
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

dev = torch.device("cuda", 0)
model, sd, _ = bench.build_model("ar354", dev)
x = torch.randn(40, 96, device=dev)
with torch.no_grad():
    for _ in range(5):
        model.log_prob(x)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t = time.perf_counter()
    pr.enable()
    for _ in range(50):
        model.log_prob(x)
    pr.disable()
    torch.cuda.synchronize()
    print("ms per step", (time.perf_counter() - t) / 50 * 1e3)
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
