"""Host-side profile (cProfile) of an NSF_AR log_prob step at its workload's
default batch (ar354: the applications' 40 rows; fe162: 50; poly2048: 40):
where the time between kernel launches goes.  usage: prof_host_ar354.py [WORKLOAD]"""
import cProfile
import pstats
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

dev = torch.device("cuda", 0)
wl = sys.argv[1] if len(sys.argv) > 1 else "ar354"
model, sd, _ = bench.build_model(wl, dev)
x = torch.randn(bench.DEFAULT_BATCH[wl], bench.WORKLOADS[wl][3], device=dev)
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
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
