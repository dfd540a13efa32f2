#!/usr/bin/env python
"""Training-step throughput (train.py:22-28: loss = -mean(prior_lp + log_det),
backward, Adam step) on one GPU, for the kernel-backed model and, beside it,
the same model run entirely through the differentiable torch restatement
(torch_math, eager torch on the same GPU), plus optionally the CPU oracle.

    python tools/bench_train.py [--workload c3] [--batch 65536] [--steps 10]

Prints one JSON line.  Not the bench.py contract line (the headline metric is
log_prob); this measures the §8(f) training row.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402  (WORKLOADS / build_model)


def torch_step_fn(model):
    from normalizingflow_amd import torch_math as tm

    def step(x):
        logdet = torch.zeros(x.shape[0], device=x.device)
        for f in model.flows:
            x, ld = tm.layer_forward(f, x, dict(f.named_parameters()), False)
            logdet = logdet + ld
        plp = model.prior.log_prob(x)
        return -torch.mean(plp + logdet)
    return step


def timed(step, opt, x, steps, warmup):
    for _ in range(warmup):
        opt.zero_grad(set_to_none=True)
        step(x).backward()
        opt.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        opt.zero_grad(set_to_none=True)
        step(x).backward()
        opt.step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3", choices=sorted(bench.WORKLOADS))
    ap.add_argument("--batch", type=int, default=1 << 16)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--cpu", action="store_true", help="also time the CPU oracle train step")
    ap.add_argument("--no-fcnn-fwd", action="store_true",
                    help="recompute forward of FCNN conditioners on library GEMMs")
    ap.add_argument("--no-train-chain", action="store_true",
                    help="one autograd node and launch per layer in the forward (config.USE_TRAIN_CHAIN off)")
    ap.add_argument("--no-fcnn-dh", action="store_true",
                    help="library GEMMs + tanh_backward for the FCNN input gradients (config.USE_FCNN_DH off)")
    ap.add_argument("--vjp-max-rows", type=int, default=None, help="override config.FUSED_VJP_MAX_ROWS")
    args = ap.parse_args()
    from normalizingflow_amd import config
    if args.vjp_max_rows is not None and hasattr(config, "FUSED_VJP_MAX_ROWS"):
        config.FUSED_VJP_MAX_ROWS = args.vjp_max_rows
    config.USE_FCNN_DH = not args.no_fcnn_dh
    config.USE_FCNN_FWD = not args.no_fcnn_fwd
    config.USE_TRAIN_CHAIN = not args.no_train_chain
    dev = torch.device("cuda", 0)
    model, sd, _ = bench.build_model(args.workload, dev)
    x = torch.randn(args.batch, bench.WORKLOADS[args.workload][3], device=dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)

    def ours(xx):
        z, plp, ld = model(xx)
        return -torch.mean(plp + ld)

    res = {"metric": "samples/sec train step (NLL fwd + bwd + Adam)", "workload": args.workload,
           "batch": args.batch, "steps": args.steps,
           "fcnn_dh": config.USE_FCNN_DH, "fcnn_fwd": config.USE_FCNN_FWD,
           "train_chain": config.USE_TRAIN_CHAIN}
    t = timed(ours, opt, x, args.steps, args.warmup)
    res["hip"] = {"ms_per_step": round(t * 1e3, 3), "samples_per_s": round(args.batch / t, 1)}
    if not args.no_torch:
        model2, _, _ = bench.build_model(args.workload, dev)
        opt2 = torch.optim.Adam(model2.parameters(), lr=1e-4)
        t2 = timed(torch_step_fn(model2), opt2, x, args.steps, args.warmup)
        res["torch_eager_same_gpu"] = {"ms_per_step": round(t2 * 1e3, 3),
                                       "samples_per_s": round(args.batch / t2, 1)}
    if args.cpu:
        from oracle import nf_oracle as orc
        specs = bench.specs_for(args.workload)
        p = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
        o = torch.optim.Adam(list(p.values()), lr=1e-4)
        n = 4096
        xc = torch.randn(n, bench.WORKLOADS[args.workload][3])
        for i in range(3):
            if i == 1:
                t0 = time.perf_counter()
            o.zero_grad()
            _, plp, ld = orc.model_forward(specs, p, xc)
            (-torch.mean(plp + ld)).backward()
            o.step()
        tc = (time.perf_counter() - t0) / 2
        res["cpu_oracle"] = {"batch": n, "ms_per_step": round(tc * 1e3, 1),
                             "samples_per_s": round(n / tc, 1), "threads": torch.get_num_threads()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
