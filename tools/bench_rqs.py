"""Microbenchmark of the streaming spline-coupling kernel (nfk_rqs_coupling) at
BASELINE c3's layer shape: B = 2^20 samples, 32 upper / 32 lower coordinates,
K = 8, NSF_CL raw conditioner logits [B, 32, 23] (param_mode 0), log|det|
accumulated.  Prints ms per launch (HIP events on the launch stream) and the
HBM rate on SURVEY 8(d)'s 3,464 algorithmic bytes per sample.

python tools/bench_rqs.py [--batch N] [--inverse] [--iters N]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from normalizingflow_amd import kernels as K_  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--inverse", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    B, n, K = args.batch, 32, 8
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, 2 * n, device=dev, generator=g)
    params = torch.randn(B, n, 3 * K - 1, device=dev, generator=g) * 0.5
    up_in = torch.arange(1, 2 * n, 2, dtype=torch.int32, device=dev)
    lo_in = torch.arange(0, 2 * n, 2, dtype=torch.int32, device=dev)
    z = torch.empty_like(x)
    ld = torch.zeros(B, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    kw = dict(lo_in=lo_in, lo_out=lo_in, logdet=ld, logdet_mode=2, K=K, left=-3.0, right=3.0,
              bottom=-3.0, top=3.0, param_mode=0, inverse=args.inverse, status=st)
    for _ in range(3):
        K_.rqs_coupling(x, params, up_in, up_in, z, **kw)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(args.iters):
        K_.rqs_coupling(x, params, up_in, up_in, z, **kw)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    byts = (2 * n * 4 + n * (3 * K - 1) * 4 + 2 * n * 4 + 8) * B
    print(json.dumps({"kernel": "nfk_rqs_coupling", "lean": os.environ.get("NFK_RQS_LEAN", "1"),
                      "inverse": args.inverse, "batch": B, "ms": round(ms, 4),
                      "GB/s": round(byts / ms / 1e6, 1), "frac_hbm": round(byts / ms / 1e6 / 8000.0, 4)}))


if __name__ == "__main__":
    main()
