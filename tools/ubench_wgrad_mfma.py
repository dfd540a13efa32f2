#!/usr/bin/env python
"""nfk_wgrad vs the split-K library GEMMs at the c3 training shapes (2^20 rows)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from normalizingflow_amd import config, fcnn_grad  # noqa: E402
from normalizingflow_amd import kernels as K_  # noqa: E402


def t_ms(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


B = 1 << 20
dev = torch.device("cuda", 0)
for M, N in ((736, 101), (100, 101), (100, 32)):
    g = torch.randn(B, M, device=dev)
    h = torch.tanh(torch.randn(B, N, device=dev))
    config.USE_WGRAD_MFMA = False
    lib = t_ms(lambda: fcnn_grad.wgrad(g, h))
    res = {"lib": lib}
    for rows in (1024, 2048, 4096, 8192):
        res["mfma_%d" % rows] = t_ms(lambda: K_.wgrad(g, h, rows_per_slice=rows))
    print("M=%d N=%d " % (M, N) + " ".join("%s %.3f ms" % kv for kv in res.items()), flush=True)
    del g, h
